#!/bin/bash
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/ncw}
mkdir -p $O
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-abft --no-latency --no-configs --config c3"
for w in ${NCWS:-6 8 10}; do
LX_LEAN_NCW=$w timeout -k 10 300 $B > $O/n$w.json 2> $O/n$w.err || exit $?
done
echo done
