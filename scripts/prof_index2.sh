#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2
CFG=${CFG:-c3}
ARGS="--config $CFG --steps 1 --warmup 0 --no-cpu --fc-queries 1048576"
P="rocprofv3 --kernel-include-regex k_index --output-format csv"
timeout -k 10 300 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/prof2/a -o a -- python3 bench.py $ARGS > gpurun_out/prof2/a.log 2>&1 || exit $?
timeout -k 10 300 $P --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR -d gpurun_out/prof2/b -o b -- python3 bench.py $ARGS > gpurun_out/prof2/b.log 2>&1 || exit $?
timeout -k 10 300 $P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/prof2/c -o c -- python3 bench.py $ARGS > gpurun_out/prof2/c.log 2>&1 || exit $?
timeout -k 10 300 $P --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum -d gpurun_out/prof2/d -o d -- python3 bench.py $ARGS > gpurun_out/prof2/d.log 2>&1 || exit $?
echo done
