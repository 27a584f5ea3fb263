#!/bin/bash
# index walk time of several builds of the library on one box (no tests: timing
# experiments may compute wrong values).  LIBS="build build_exp ..." CFGS="c3"
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/libs}
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-abft --no-latency --no-configs"
for cfg in ${CFGS:-c3}; do
for rep in 1 2; do
for v in ${LIBS:-build build_old}; do
export LX_LIB=$PWD/lachesis-base_amd/$v/liblachesis_hip.so
timeout -k 10 300 $B --config $cfg $EXTRA > $O/${cfg}_${v}_$rep.json 2> $O/${cfg}_${v}_$rep.err || exit $?
python3 -c "import json; d=json.load(open('$O/${cfg}_${v}_$rep.json')); print('$cfg $v $rep', round(d['index_kernel_ms'],2), 'ms')"
done
done
done
echo done
