set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_head
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/feed -o feed -- python3 scripts/feed_probe.py > $O/feed.json 2> $O/feed.err || exit $?
timeout -k 10 600 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
tail -c 400 $O/bench_default.json
OUT=$O/prof bash scripts/prof_round.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/abft_trace -o at -- python3 scripts/bench_abft_only.py 2 > $O/abft_trace.log 2>&1 || exit $?
echo done
