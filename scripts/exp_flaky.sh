#!/bin/bash
# repeat the fork-DAG multi-batch parity test with build/ and build_old/
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/flaky}
mkdir -p $O
for v in new old; do
if [ $v = old ]; then export LX_LIB=$PWD/lachesis-base_amd/build_old/liblachesis_hip.so; else unset LX_LIB; fi
for rep in 1 2 3; do
timeout -k 10 200 python3 -u -m pytest -q --timeout 100 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "config4_scaled or fork_dag or batching" > $O/${v}_$rep.log 2>&1
rc=$?
echo "$v $rep rc=$rc $(tail -n 1 $O/${v}_$rep.log)"
[ $rc -le 1 ] || exit $rc
done
done
echo done
