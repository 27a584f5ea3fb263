#!/bin/bash
# Per-rank compute of a G-way column shard, measured alone on one GPU
# (bench.py --shard-solo G): rank 0's index walk over its columns + packing of
# its outgoing LowestAfter blocks, and its partial ForklessCause.  What the
# N-GPU run adds on top is the RCCL all-to-all / all-reduce over xGMI.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for G in ${GS:-2 4 8}; do
  timeout -k 10 300 python bench.py --shard-solo $G --no-cpu --no-abft --no-latency --no-configs --steps 3 --warmup 1 \
     > gpurun_out/solo_g$G.log 2>&1 || { echo "G=$G rc=$?"; tail -5 gpurun_out/solo_g$G.log; exit 1; }
  tail -1 gpurun_out/solo_g$G.log
done
