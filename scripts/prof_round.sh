#!/bin/bash
# Profile evidence for profiles/<round>/: rocprofv3 kernel stats of the
# default bench run (all legs but the CPU baselines), then k_index / k_fc HBM
# traffic of the headline config alone from PMC passes (one TCC counter group
# per pass, as MI355X_MICROARCH.md prescribes), converted by
# scripts/traffic_json.py.
#   OUT=gpurun_out/prof_r03 bash scripts/prof_round.sh
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/prof_round}
mkdir -p $O
if [ -z "$PMC_ONLY" ]; then   # PMC_ONLY=1: the counter passes alone
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --no-cpu --no-power > $O/kt.log 2>&1 || exit $?
python3 scripts/headline_kernels.py $O/kt > $O/headline_kernels.json || exit $?
fi
[ -n "$NO_PMC" ] && { find $O -name "*trace*.csv" -delete; echo done; exit 0; }   # NO_PMC=1: the kernel stats alone
A="--config ${CFG:-c3} --steps 2 --warmup 1 --no-cpu --no-power --no-abft --no-latency --no-configs --no-dropin"
P="rocprofv3 --kernel-include-regex k_fc|k_index --output-format csv"
timeout -k 10 300 $P --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ -d $O/rdreq -o rdreq -- python3 bench.py $A > $O/rdreq.log 2>&1 || exit $?
timeout -k 10 300 $P --pmc WRITE_SIZE TCC_EA0_WRREQ TCC_EA0_WRREQ_64B -d $O/write -o write -- python3 bench.py $A > $O/write.log 2>&1 || exit $?
timeout -k 10 300 $P --pmc FETCH_SIZE -d $O/fetch -o fetch -- python3 bench.py $A > $O/fetch.log 2>&1 || exit $?
python3 scripts/traffic_json.py $O > $O/traffic_${CFG:-c3}.json || exit $?
find $O -name "*trace*.csv" -delete
echo done
