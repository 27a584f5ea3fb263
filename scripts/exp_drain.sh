#!/bin/bash
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/drain}
mkdir -p $O
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-abft --no-latency --no-configs --config c3"
export LX_WALKER=block LX_LEAN_NCW=8
timeout -k 10 300 $B > $O/fill.json 2> $O/fill.err || exit $?
LX_DIAG_NOFILL=1 timeout -k 10 300 $B > $O/nofill.json 2> $O/nofill.err || exit $?
echo done
