set -o pipefail
bash scripts/probes/r06_call11.sh || exit $?
O=gpurun_out/r06_evict2
mkdir -p $O
for i in 1 2 3; do
  WM_INST=1 WM_WALKS=4 timeout -k 10 200 python3 scripts/probes/walk_modes2.py >> $O/walks.jsonl 2>> $O/walks.err || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r06_evict2/walks.jsonl"):
    d = json.loads(l)
    print(d["walk_ms"], [sum(v["evicted_ms"] for v in k.values()) for k in d.get("kfd_delta", [])])
PY
