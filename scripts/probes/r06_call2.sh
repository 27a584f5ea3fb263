set -o pipefail
bash scripts/probes/power_ab_r06.sh; echo "power rc=$?"
mkdir -p gpurun_out/r06_t2
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_shard_dropin.py > gpurun_out/r06_t2/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r06_t2/pytest.log; exit $rc
