#!/bin/bash
# the fork-DAG multi-batch parity tests with each build variant
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/flaky2}
mkdir -p $O
for v in build build_NOMAX3 build_NOBIT31; do
export LX_LIB=$PWD/lachesis-base_amd/$v/liblachesis_hip.so
timeout -k 10 200 python3 -u -m pytest -q --timeout 100 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "config4_scaled or batching" > $O/$v.log 2>&1
rc=$?
echo "$v rc=$rc $(tail -n 1 $O/$v.log)"
[ $rc -le 1 ] || exit $rc
done
echo done
