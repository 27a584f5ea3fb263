#!/bin/bash
# PMC passes on the index walker (k_index): instruction mix, waits, LDS, L2/HBM.
# Usage: CFG=c3 TAG=v7 bash scripts/prof_index2.sh
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
CFG=${CFG:-c3}
TAG=${TAG:-cur}
O=gpurun_out/pmc_${TAG}_${CFG}
mkdir -p $O
ARGS="--config $CFG --steps 1 --warmup 0 --no-cpu --fc-queries 1048576"
P="rocprofv3 --kernel-include-regex k_index --output-format csv"
timeout -k 10 300 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/a -o a -- python3 bench.py $ARGS > $O/a.log 2>&1 || exit $?
timeout -k 10 300 $P --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR -d $O/b -o b -- python3 bench.py $ARGS > $O/b.log 2>&1 || exit $?
timeout -k 10 300 $P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d $O/c -o c -- python3 bench.py $ARGS > $O/c.log 2>&1 || exit $?
echo done
