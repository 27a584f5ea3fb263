set -o pipefail
mkdir -p gpurun_out/r06_t1
bash scripts/probes/clock_power_r06.sh; echo "clkpow rc=$?"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_fc_early.py tests/test_gpu_getsrv.py tests/test_gpu_shard_dist.py tests/test_gpu_shard_dropin.py > gpurun_out/r06_t1/pytest.log 2>&1
rc=$?; tail -30 gpurun_out/r06_t1/pytest.log; exit $rc
