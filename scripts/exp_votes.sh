#!/bin/bash
# abft: GPU tests with the tiled vote kernel, then C5 timing vs the one-voter kernel
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/votes}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_abft.py -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python3 scripts/bench_abft_only.py 5 > $O/tile.json 2> $O/tile.err || exit $?
LX_VOTE_ONE=1 timeout -k 10 200 python3 scripts/bench_abft_only.py 5 > $O/one.json 2> $O/one.err || exit $?
echo done
