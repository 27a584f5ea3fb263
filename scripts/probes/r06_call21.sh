set -o pipefail
OUT=gpurun_out/r06_tests_final2 bash scripts/gpu_tests.sh || { tail -30 gpurun_out/r06_tests_final2/pytest.log; exit 1; }
tail -1 gpurun_out/r06_tests_final2/pytest.log
bash scripts/probes/r06_call20.sh
