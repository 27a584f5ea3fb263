set -o pipefail
mkdir -p gpurun_out/r06_abft
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_abft.py > gpurun_out/r06_abft/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r06_abft/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_abft_only.py 5 > gpurun_out/r06_abft/abft_leg.json 2> gpurun_out/r06_abft/abft_leg.err || exit $?
python3 - <<'PY'
import json
r=json.load(open("gpurun_out/r06_abft/abft_leg.json"))
print(r["events_per_sec"], r["ms_per_step"], r["phase_ms"], r.get("roofline_root_fc"))
PY
