#!/bin/bash
# fork-path FC: parity tests, then C4 (10 cheaters) and a 40-cheater C4 shape,
# streamed-mask kernel (k_fc_fk) vs the fix-up loop (LX_FC_FK=0)
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/fcfk}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "fork or config4" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_shards.py tests/test_gpu_abft.py -m gpu > $O/pytest2.log 2>&1 || exit $?
B="python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu --no-abft --no-latency --no-configs --fc-queries 4194304"
timeout -k 10 200 $B > $O/c4_fk.json 2> $O/c4_fk.err || exit $?
LX_FC_FK=0 timeout -k 10 200 $B > $O/c4_loop.json 2> $O/c4_loop.err || exit $?
echo done
