#!/bin/bash
# LDS occupancy of the shipped C3 walk (k_index_segs): bank conflicts, LDS-array
# cycles, LDS issue stalls and the instruction mix, two separate --pmc passes.
#   OUT=gpurun_out/wlds bash scripts/walker_lds_pmc.sh
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/wlds}
mkdir -p $O
B="python3 bench.py --config ${CFG:-c3} --steps 1 --warmup 0 --no-cpu --no-abft --no-dropin --no-latency --no-configs --fc-queries 1048576"
P="rocprofv3 --kernel-include-regex k_index --output-format csv"
timeout -s KILL 240 $P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/a -o a -- $B > $O/a.log 2>&1 || exit $?
timeout -s KILL 240 $P --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d $O/b -o b -- $B > $O/b.log 2>&1 || exit $?
find $O -name "*trace*.csv" -delete
echo done
