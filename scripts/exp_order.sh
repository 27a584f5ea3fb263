#!/bin/bash
# index walk time with the batch in generator (Add) order vs level order
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/order}
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-abft --no-latency --no-configs"
for cfg in ${CFGS:-c3}; do
for ord in add level; do
timeout -k 10 300 $B --config $cfg --order $ord $EXTRA > $O/${cfg}_${ord}.json 2> $O/${cfg}_${ord}.err || exit $?
python3 -c "import json; d=json.load(open('$O/${cfg}_${ord}.json')); print('$cfg $ord', round(d['index_kernel_ms'],2), 'ms', round(d['value']/1e6,1), 'M ev/s', round(d['fc_queries_per_sec']/1e9,3), 'G q/s')"
done
done
echo done
