#!/bin/bash
# Column-shard rehearsal on ONE GPU: G ranks share cuda:0 over gloo (staged
# collectives), so kernel times per rank are indicative, collective times are
# not (the driver's N>1 runs use RCCL over xGMI, one GPU per rank).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp LX_DIST_BACKEND=gloo
for G in ${GS:-2 4}; do
  timeout -k 10 ${T:-400} python -m torch.distributed.run --nnodes=1 --nproc-per-node $G --master-addr 127.0.0.1 \
     --master-port $((29500 + G)) bench.py --gpus $G --mode shard ${ARGS:---no-cpu --no-abft --steps 2 --warmup 1} \
     > gpurun_out/shard_g$G.log 2>&1 || { echo "G=$G failed rc=$?"; tail -20 gpurun_out/shard_g$G.log; exit 1; }
  tail -1 gpurun_out/shard_g$G.log
done
