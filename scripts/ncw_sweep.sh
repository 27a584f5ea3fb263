#!/bin/bash
# k_index compute-wave count sweep (LX_NCW) at the default CPW.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for c in ${NCWS:-4 2 1}; do
  LX_NCW=$c timeout -k 10 300 python bench.py --no-cpu --no-abft --steps 2 --warmup 1 ${ARGS} > gpurun_out/ncw$c.log 2>&1 || { echo "ncw=$c rc=$?"; tail -5 gpurun_out/ncw$c.log; exit 1; }
  echo "ncw=$c $(tail -1 gpurun_out/ncw$c.log | python3 -c 'import sys,json; j=json.loads(sys.stdin.read()); print("k_index_ms=%.1f step_ms=%.1f" % (j["index_kernel_ms"], j["ms_per_step"]))')"
done
