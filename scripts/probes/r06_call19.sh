set -o pipefail
OUT=gpurun_out/r06_tests_stage bash scripts/gpu_tests.sh || { tail -30 gpurun_out/r06_tests_stage/pytest.log; exit 1; }
tail -1 gpurun_out/r06_tests_stage/pytest.log
bash scripts/probes/r06_call11.sh
