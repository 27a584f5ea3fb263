set -o pipefail
O=gpurun_out/r06_alt
mkdir -p $O
for i in 1 2; do
  WA_ROUNDS=4 timeout -k 10 240 python3 scripts/probes/walk_alt.py >> $O/alt.jsonl 2>> $O/alt.err || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r06_alt/alt.jsonl"):
    d = json.loads(l)
    print(d["pid"], d["round"], d["handle"], d["walk_ms"], d["walk_ms_by_segment"], d["mhz"], d["evicted_ms"])
PY
