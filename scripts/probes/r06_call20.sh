set -o pipefail
O=gpurun_out/r06_final
mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log > $O/bench_default.json
OUT=$O/prof NO_PMC=1 bash scripts/prof_round.sh || exit $?
cp $O/prof/headline_kernels.json $O/
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_final/bench_default.json").read())
print(d["value"], d["ms_per_step"], d.get("walk_clock", {}).get("mhz_median"), d["roofline"]["frac"], d["abft"]["events_per_sec"])
PY
