set -o pipefail
mkdir -p gpurun_out/r06_margin
for i in 1 2; do
  WL_OPT=drain_margin WL_VALUES=0,1024,512 WL_ROUNDS=3 timeout -k 10 300 python3 scripts/probes/walk_lock_ab.py >> gpurun_out/r06_margin/margin_ab.jsonl 2>> gpurun_out/r06_margin/ab.err || exit $?
  WL_OPT=pad_slice WL_VALUES=0,1 WL_ROUNDS=3 timeout -k 10 300 python3 scripts/probes/walk_lock_ab.py >> gpurun_out/r06_margin/pad_ab.jsonl 2>> gpurun_out/r06_margin/ab.err || exit $?
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread "tests/test_gpu_parity.py::test_config3_shape_1m_default_segments_vs_oracle" "tests/test_gpu_parity.py::test_walker_variants" > gpurun_out/r06_margin/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r06_margin/pytest.log; exit $rc
