#!/bin/bash
# k_index columns-per-workgroup sweep on the unsharded C3 index (LX_CPW).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for c in ${CPWS:-4 2 1}; do
  LX_CPW=$c timeout -k 10 300 python bench.py --no-cpu --no-abft --steps 2 --warmup 1 ${ARGS} > gpurun_out/cpw$c.log 2>&1 || { echo "cpw=$c rc=$?"; tail -5 gpurun_out/cpw$c.log; exit 1; }
  echo "cpw=$c $(tail -1 gpurun_out/cpw$c.log | python3 -c 'import sys,json; j=json.loads(sys.stdin.read()); print("k_index_ms=%.1f step_ms=%.1f" % (j["index_kernel_ms"], j["ms_per_step"]))')"
done
