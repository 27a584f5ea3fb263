#!/bin/bash
# rocprofv3 passes on the index walker (kernel trace + PMC, separate passes).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
CFG=${CFG:-c2}
ARGS="--config $CFG --steps 1 --warmup 0 --no-cpu --fc-queries 1048576"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "k_index" -d gpurun_out/prof/pmc1 -o pmc1 --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --kernel-include-regex "k_index" -d gpurun_out/prof/pmc2 -o pmc2 --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/pmc2.log 2>&1 || exit $?
echo done
