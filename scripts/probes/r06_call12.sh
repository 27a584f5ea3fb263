set -o pipefail
O=gpurun_out/r06_fc16pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="rocprofv3 --kernel-include-regex k_root_fc16 --output-format csv"
timeout -s KILL 120 $P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/p1 -o p1 -- python3 scripts/bench_abft_only.py 2 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 $P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES -d $O/p2 -o p2 -- python3 scripts/bench_abft_only.py 2 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
find $O -name "*counter_collection.csv" | head
