#!/bin/bash
# block walker: parity of the walker variants, timing of drain / wave configurations, counters
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/block}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "walker" > $O/pytest.log 2>&1 || exit $?
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-abft --no-latency --no-configs --config c3"
for v in ${VARS:-8:2 8:4 11:4}; do
N=${v%%:*}; D=${v##*:}
LX_WALKER=block LX_LEAN_NCW=$N LX_DRAINS=$D timeout -k 10 300 $B > $O/b${N}_d$D.json 2> $O/b${N}_d$D.err || exit $?
done
export LX_LIB=$PWD/lachesis-base_amd/build_wprof/liblachesis_hip.so LX_PROF=1
for v in ${PVARS:-8:2 8:4}; do
N=${v%%:*}; D=${v##*:}
LX_WALKER=block LX_LEAN_NCW=$N LX_DRAINS=$D timeout -k 10 300 python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu --no-abft --no-latency --no-configs > $O/p${N}_d$D.json 2> $O/p${N}_d$D.err || exit $?
done
echo done
