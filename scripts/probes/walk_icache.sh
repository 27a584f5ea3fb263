#!/bin/bash
# Fast / slow walk modes under the instruction-fetch counters: N walk_time.py
# processes in a row, each under one rocprofv3 --pmc pass.
#   OUT=gpurun_out/wic N=4 bash scripts/probes/walk_icache.sh
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/wic}
mkdir -p $O
C="${CTRS:-SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE}"
for i in $(seq 1 ${N:-4}); do
  timeout -k 10 240 rocprofv3 --kernel-include-regex k_index --output-format csv --pmc $C -d $O/p$i -o p$i -- \
      python3 scripts/probes/walk_time.py > $O/p$i.log 2>&1 || exit $?
  tail -n 1 $O/p$i.log
done
find $O -name "*trace*.csv" -delete
