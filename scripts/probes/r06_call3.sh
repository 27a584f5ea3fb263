set -o pipefail
# power of the walk (shipped / no LA stores / no HB stores)
bash scripts/probes/power_ab_r06.sh; echo "power rc=$?"
# seg_xmap A/B: the shipped build with option seg_xmap=1 against its default, processes alternating
OUT=gpurun_out/r06_xmap R=3 AB_OPTS='{"seg_xmap": 1}' bash scripts/probes/walk_ab.sh > /dev/null; echo "xmap ab rc=$?"
export TMPDIR=/tmp
for X in 0 1; do
  WT_OPTS="{\"seg_xmap\": $X}" WM_INST=1 WM_WALKS=2 timeout -s KILL 180 rocprofv3 --kernel-include-regex k_index --output-format csv \
    --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_WRREQ_STALL TCC_EA0_RDREQ -d gpurun_out/r06_xmap/pmc_x$X -o p \
    -- python3 scripts/probes/walk_modes2.py > gpurun_out/r06_xmap/pmc_x$X.log 2>&1 || exit $?
done
mkdir -p gpurun_out/r06_t3
timeout -k 10 1200 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_shard_dropin.py "tests/test_gpu_parity.py::test_config3_shape_1m_default_segments_vs_oracle" > gpurun_out/r06_t3/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r06_t3/pytest.log; exit $rc
