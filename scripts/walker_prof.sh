#!/bin/bash
# k_index per-wave counters and per-segment cycles (make wprof build).
#   OUT=gpurun_out/wprof CFGS="c3 c2" bash scripts/walker_prof.sh   
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/wprof}
mkdir -p $O
export LX_LIB=$PWD/lachesis-base_amd/build_wprof/liblachesis_hip.so LX_PROF=1
for c in ${CFGS:-c3 c2}; do
timeout -k 10 300 python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu --no-abft --no-latency --no-configs > $O/$c.json 2> $O/$c.err || exit $?
done
grep -h "lx_prof" $O/*.err | head -40
