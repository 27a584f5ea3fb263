#!/bin/bash
# block walker on 1/2/4-column slices: parity (walker tests, shards), then
# index timing: C2 (V=100), C4, and a C3 column shard of G=2/4/8 alone
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/cpw}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "walker or fork or config" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_shards.py -m gpu > $O/pytest_shards.log 2>&1 || exit $?
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-abft --no-latency --no-configs"
for cfg in c2 c4; do
for c in 4 auto; do
if [ $c = auto ]; then unset LX_CPW; else export LX_CPW=$c; fi
timeout -k 10 300 $B --config $cfg > $O/${cfg}_$c.json 2> $O/${cfg}_$c.err || exit $?
python3 -c "import json; d=json.load(open('$O/${cfg}_$c.json')); print('$cfg cpw $c', round(d['index_kernel_ms'],2), 'ms', round(d['value']/1e6,2), 'M ev/s')"
done
done
unset LX_CPW
for g in 8 4 2; do
for c in 4 auto; do
if [ $c = auto ]; then unset LX_CPW; else export LX_CPW=$c; fi
timeout -k 10 300 $B --config c3 --shard-solo $g > $O/solo${g}_$c.json 2> $O/solo${g}_$c.err || exit $?
python3 -c "import json; d=json.load(open('$O/solo${g}_$c.json')); print('solo $g cpw $c', {k: v for k, v in d.items() if 'ms' in k})"
done
done
echo done
