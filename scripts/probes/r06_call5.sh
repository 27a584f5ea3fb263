set -o pipefail
mkdir -p gpurun_out/r06_skew2 gpurun_out/r06_bench
for i in 1 2; do
LX_LIB=lachesis-base_amd/build_pSKEW/liblachesis_hip.so WS_WALKS=2 timeout -k 10 240 python3 scripts/probes/walk_skew.py >> gpurun_out/r06_skew2/skew.jsonl 2>> gpurun_out/r06_skew2/skew.err || exit $?
done
timeout -k 10 900 python3 bench.py > gpurun_out/r06_bench/bench_default.log 2>&1; rc=$?
tail -c 600 gpurun_out/r06_bench/bench_default.log; exit $rc
