#!/bin/bash
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/knobs}
mkdir -p $O
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-abft --no-latency --no-configs --config c3"
for d in ${DIAGS:-0 16 32 48}; do
LX_DIAG=$d timeout -k 10 300 $B > $O/d$d.json 2> $O/d$d.err || exit $?
done
echo done
