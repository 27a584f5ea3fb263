#!/bin/bash
# block walker on the other shapes: C2 (V=100), a 1/8 column shard of C3, abft C5
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/block2}
mkdir -p $O
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-abft --no-latency --no-configs"
BL="LX_WALKER=block LX_LEAN_NCW=8 LX_DRAINS=4 LX_CPW=4"
timeout -k 10 300 $B --config c2 > $O/c2_base.json 2> $O/c2_base.err || exit $?
env $BL timeout -k 10 300 $B --config c2 > $O/c2_block.json 2> $O/c2_block.err || exit $?
timeout -k 10 300 $B --config c3 --shard-solo 8 > $O/s8_base.json 2> $O/s8_base.err || exit $?
env $BL timeout -k 10 300 $B --config c3 --shard-solo 8 > $O/s8_block.json 2> $O/s8_block.err || exit $?
timeout -k 10 200 python3 scripts/bench_abft_only.py 5 > $O/c5_base.json 2> $O/c5_base.err || exit $?
env $BL timeout -k 10 200 python3 scripts/bench_abft_only.py 5 > $O/c5_block.json 2> $O/c5_block.err || exit $?
echo done
