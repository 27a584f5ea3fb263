#!/bin/bash
# index walk time under several runtime knob settings on one box (timing only).
#   ENVS="base|LX_DRAINS=2|LX_DIAG=32" CFGS="c3" bash scripts/exp_env.sh
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/env}
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-abft --no-latency --no-configs"
IFS='|' read -ra VS <<< "${ENVS:-base}"
for cfg in ${CFGS:-c3}; do
for rep in 1 2; do
i=0
for v in "${VS[@]}"; do
i=$((i+1))
if [ "$v" = base ]; then E=""; else E="$v"; fi
timeout -k 10 300 env $E $B --config $cfg $EXTRA > $O/${cfg}_${i}_$rep.json 2> $O/${cfg}_${i}_$rep.err || exit $?
python3 -c "import json; d=json.load(open('$O/${cfg}_${i}_$rep.json')); print('$cfg [$v] $rep', round(d['index_kernel_ms'],2), 'ms')"
done
done
done
echo done
