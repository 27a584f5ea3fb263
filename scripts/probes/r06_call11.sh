set -o pipefail
O=gpurun_out/r06_abfttime
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_abft.py tests/test_gpu_fccache.py tests/test_gpu_dropin.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit $rc
LX_ABFT_TIMING=1 timeout -k 10 200 python3 scripts/bench_abft_only.py 4 > $O/leg.json 2> $O/timing.err || exit $?
grep abft_timing $O/timing.err | tail -6
cut -c1-400 $O/leg.json
