#!/bin/bash
# HBM traffic of k_fc / k_index per launch from PMC counters, collected as
# MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes (TCC slots), FETCH_SIZE doubled on gfx950 for 16-B-per-lane
# streaming reads.  Output: gpurun_out/traffic/{fetch,write}/... CSVs.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/traffic
mkdir -p $O
ARGS="${ARGS:---config c3 --steps 2 --warmup 1 --no-cpu}"
P="rocprofv3 --kernel-include-regex k_fc|k_index --output-format csv"
timeout -k 10 400 $P --pmc FETCH_SIZE -d $O/fetch -o fetch -- python3 bench.py $ARGS > $O/fetch.log 2>&1 || exit $?
timeout -k 10 400 $P --pmc WRITE_SIZE -d $O/write -o write -- python3 bench.py $ARGS > $O/write.log 2>&1 || exit $?
echo done
