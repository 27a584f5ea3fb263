#!/bin/bash
# fork-path FC: parity tests that cover cheaters, then the C4 line
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/fc4}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_small.py -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-abft --no-latency --no-configs > $O/c4.json 2> $O/c4.err || exit $?
echo done
