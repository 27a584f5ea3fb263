#!/bin/bash
# lean walker A/B: parity tests of the walker variants, then index timing.
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/lean}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "walker" > $O/pytest.log 2>&1 || exit $?
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-abft --no-latency --no-configs"
for cfg in ${CFGS:-c3 c4}; do
timeout -k 10 300 $B --config $cfg > $O/${cfg}_base.json 2> $O/${cfg}_base.err || exit $?
for v in ${VARS:-lean:8 block:8}; do
W=${v%%:*}; N=${v##*:}
LX_WALKER=$W LX_LEAN_NCW=$N timeout -k 10 300 $B --config $cfg > $O/${cfg}_$W$N.json 2> $O/${cfg}_$W$N.err || exit $?
done
done
if [ -n "$PROF" ]; then
export LX_LIB=$PWD/lachesis-base_amd/build_wprof/liblachesis_hip.so LX_PROF=1
for v in ${VARS:-lean:8 block:8}; do
W=${v%%:*}; N=${v##*:}
LX_WALKER=$W LX_LEAN_NCW=$N timeout -k 10 300 python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu --no-abft --no-latency --no-configs > $O/prof$W$N.json 2> $O/prof$W$N.err || exit $?
grep lx_prof $O/prof$W$N.err | head -2
done
fi
echo done
