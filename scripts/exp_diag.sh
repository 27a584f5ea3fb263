#!/bin/bash
# walker A/B over LX_DIAG bits (same box, interleaved), plus the fill-disabled walk
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/diag}
mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "walker" > $O/pytest.log 2>&1 || exit $?
fi
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-abft --no-latency --no-configs --config ${CFG:-c3}"
for rep in 1 2; do
for d in ${DIAGS:-0 64 128 192}; do
LX_DIAG=$d timeout -k 10 300 $B > $O/d${d}_$rep.json 2> $O/d${d}_$rep.err || exit $?
python3 -c "import json,sys; d=json.load(open('$O/d${d}_$rep.json')); print('diag $d rep $rep', round(d['index_kernel_ms'],2), 'ms')"
done
done
if [ -n "$NOFILL" ]; then
LX_DIAG_NOFILL=1 timeout -k 10 300 $B > $O/nofill.json 2> $O/nofill.err || exit $?
python3 -c "import json,sys; d=json.load(open('$O/nofill.json')); print('nofill', round(d['index_kernel_ms'],2), 'ms')"
fi
echo done
