#!/bin/bash
# C3 unsharded: block walker on 4-column slices (one workgroup per CU) vs
# 2-column slices with a 512-record ring (two workgroups per CU)
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/c3cpw2}
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-abft --no-latency --no-configs --config c3"
for v in base rr512d4 rr512d2 base; do
case $v in
base) E="" ;;
rr512d4) E="LX_CPW=2 LX_RR=512" ;;
rr512d2) E="LX_CPW=2 LX_RR=512 LX_DRAINS=2" ;;
esac
env $E timeout -k 10 300 $B > $O/$v.json 2> $O/$v.err || exit $?
python3 -c "import json; d=json.load(open('$O/$v.json')); print('$v', round(d['index_kernel_ms'],2), 'ms')"
done
echo done
