#!/bin/bash
# Profile evidence for profiles/<round>/: rocprofv3 kernel stats of the default
# bench line, then HBM traffic of k_fc / k_index from PMC counters collected
# as MI355X_MICROARCH.md prescribes (FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes), converted by scripts/traffic_json.py.
#   OUT=gpurun_out/prof_r01 bash scripts/prof_round.sh
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/prof_round}
mkdir -p $O
ARGS="${ARGS:---config c3 --steps 3 --warmup 1 --no-cpu}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $ARGS --no-abft > $O/kt.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_abft -o kt_abft -- python3 scripts/bench_abft_only.py > $O/kt_abft.log 2>&1 || exit $?
P="rocprofv3 --kernel-include-regex k_fc|k_index --output-format csv"
timeout -k 10 400 $P --pmc FETCH_SIZE -d $O/fetch -o fetch -- python3 bench.py $ARGS --no-abft > $O/fetch.log 2>&1 || exit $?
timeout -k 10 400 $P --pmc WRITE_SIZE -d $O/write -o write -- python3 bench.py $ARGS --no-abft > $O/write.log 2>&1 || exit $?
python3 scripts/traffic_json.py $O > $O/traffic_c3.json || exit $?
echo done
