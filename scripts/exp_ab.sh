#!/bin/bash
# same-box A/B of the library in build/ against build_old/ (index walk timing),
# after the walker parity tests of the new build
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/ab}
mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "walker or fork_dag or config" > $O/pytest.log 2>&1 || exit $?
fi
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-abft --no-latency --no-configs"
for cfg in ${CFGS:-c3}; do
for rep in 1 2; do
for v in new old; do
if [ $v = old ]; then export LX_LIB=$PWD/lachesis-base_amd/build_old/liblachesis_hip.so; else unset LX_LIB; fi
timeout -k 10 300 $B --config $cfg $EXTRA > $O/${cfg}_${v}_$rep.json 2> $O/${cfg}_${v}_$rep.err || exit $?
python3 -c "import json; d=json.load(open('$O/${cfg}_${v}_$rep.json')); print('$cfg $v $rep', round(d['index_kernel_ms'],2), 'ms')"
done
done
done
echo done
