#!/bin/bash
# abft (BASELINE configs[4]) evidence: GPU abft tests, the abft leg's timing,
# rocprofv3 kernel stats (launch / copy counts per epoch), and VALU counters of
# k_root_fc in separate --pmc passes (PMC=1).
#   OUT=gpurun_out/abft bash scripts/prof_abft.sh
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/prof_abft}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_abft.py -m gpu > $O/pytest_abft.log 2>&1 || exit $?
timeout -k 10 200 python3 scripts/bench_abft_only.py 5 > $O/abft.json 2> $O/abft.err || exit $?
LX_ABFT_TRACE=1 timeout -k 10 200 python3 scripts/bench_abft_only.py 1 > $O/trace.json 2> $O/trace.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/kt -o kt -- python3 scripts/bench_abft_only.py 5 > $O/kt.log 2>&1 || exit $?
if [ -n "$PMC" ]; then
P="rocprofv3 --kernel-include-regex k_root_fc --output-format csv"
timeout -s KILL 120 $P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $O/pmc1 -o pmc1 -- python3 scripts/bench_abft_only.py 2 > $O/pmc1.log 2>&1 || exit $?
timeout -s KILL 120 $P --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc2 -o pmc2 -- python3 scripts/bench_abft_only.py 2 > $O/pmc2.log 2>&1 || exit $?
fi
find $O -name "*trace*.csv" -delete
echo done
