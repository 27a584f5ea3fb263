set -o pipefail
O=gpurun_out/r06_move
mkdir -p $O
for i in 1 2 3; do
  WA_MOVE=1 WA_ROUNDS=6 timeout -k 10 240 python3 scripts/probes/walk_alt.py >> $O/alt.jsonl 2>> $O/alt.err || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r06_move/alt.jsonl"):
    d = json.loads(l)
    print(d["pid"], d["round"], d["handle"], d["moved"], d["walk_ms"], d["mhz"])
PY
