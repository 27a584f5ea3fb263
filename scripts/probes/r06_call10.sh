set -o pipefail
O=gpurun_out/r06_abftprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 scripts/bench_abft_only.py 5 > $O/leg.json 2> $O/leg.err || exit $?
find $O/kt -name "*kernel_stats.csv" | head -3
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; head -30 $O/kernel_stats.csv | cut -c1-200
