#!/bin/bash
# k_index issue / LDS / instruction-cache counters (separate --pmc passes, kernel filter).
#   OUT=gpurun_out/wpmc CFG=c3 bash scripts/walker_pmc.sh     (LX_* env passes through)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/wpmc}
mkdir -p $O
CFG=${CFG:-c3}
B="python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu --no-abft --no-latency --no-configs"
P="rocprofv3 --kernel-include-regex k_index --output-format csv"
timeout -s KILL 200 $P --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH SQ_INSTS_BRANCH SQC_ICACHE_HITS SQC_ICACHE_MISSES GRBM_GUI_ACTIVE -d $O/p1 -o p1 -- $B > $O/p1.log 2>&1 || exit $?
timeout -s KILL 200 $P --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/p2 -o p2 -- $B > $O/p2.log 2>&1 || exit $?
find $O -name "*trace*.csv" -delete
echo done
