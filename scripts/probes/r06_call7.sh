set -o pipefail
mkdir -p gpurun_out/r06_crec
for i in 1 2 3; do
  WL_OPT=crec WL_VALUES=0,1 WL_ROUNDS=4 timeout -k 10 300 python3 scripts/probes/walk_lock_ab.py >> gpurun_out/r06_crec/crec_ab.jsonl 2>> gpurun_out/r06_crec/crec_ab.err || exit $?
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread "tests/test_gpu_parity.py::test_config3_shape_1m_default_segments_vs_oracle" > gpurun_out/r06_crec/pytest.log 2>&1
rc=$?; tail -8 gpurun_out/r06_crec/pytest.log; exit $rc
