#!/bin/bash
# One round-validation GPU call: GPU tests + smoke, the level-fed probe under
# rocprofv3 (k_small), the default bench line, then rocprof kernel stats and
# the PMC traffic passes (scripts/prof_round.sh).
#   OUT=gpurun_out/r03_head bash scripts/round_check.sh
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/round_check}
mkdir -p $O
OUT=$O/tests bash scripts/gpu_tests.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/feed -o feed -- python3 scripts/feed_probe.py > $O/feed.json 2> $O/feed.err || exit $?
[ -n "$QUICK" ] && exit 0
timeout -k 10 600 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
OUT=$O/prof bash scripts/prof_round.sh || exit $?
echo done
