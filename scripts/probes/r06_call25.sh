set -o pipefail
# the record-move probe on whatever box comes up (looking for one in the
# walk's slow mode)
O=gpurun_out/r06_move_$(date +%s)
mkdir -p $O
for i in 1 2; do
  WA_MOVE=1 WA_ROUNDS=6 timeout -k 10 240 python3 scripts/probes/walk_alt.py >> $O/alt.jsonl 2>> $O/alt.err || exit $?
done
python3 - "$O" <<'PY'
import json, sys
for l in open(sys.argv[1] + "/alt.jsonl"):
    d = json.loads(l)
    print(d["pid"], d["round"], d["handle"], d["moved"], d["walk_ms"], d["mhz"])
PY
