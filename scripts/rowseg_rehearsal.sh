#!/bin/bash
# Row-segment rehearsal on ONE GPU: G ranks share cuda:0 over gloo (staged
# collectives), so each rank's walk runs concurrently with the others' on the
# same GPU and the collective times are host staging; the driver's N>1 runs
# use RCCL over xGMI, one GPU per rank.  Checks the protocol at full size.
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out}
mkdir -p $O
export TMPDIR=/tmp LX_DIST_BACKEND=gloo
for G in ${GS:-2}; do
  timeout -k 10 ${T:-400} python -m torch.distributed.run --nnodes=1 --nproc-per-node $G --master-addr 127.0.0.1 \
     --master-port $((29600 + G)) bench.py --gpus $G --mode rowseg ${ARGS:---no-cpu --no-abft --steps 2 --warmup 1} \
     > $O/rowseg_g$G.log 2>&1 || { echo "G=$G failed rc=$?"; tail -20 $O/rowseg_g$G.log; exit 1; }
  tail -1 $O/rowseg_g$G.log
done
