set -o pipefail
mkdir -p gpurun_out/r06_skew3
for i in 1 2 3; do
LX_LIB=lachesis-base_amd/build_pSKEW/liblachesis_hip.so WS_WALKS=2 timeout -k 10 240 python3 scripts/probes/walk_skew.py >> gpurun_out/r06_skew3/skew.jsonl 2>> gpurun_out/r06_skew3/skew.err || exit $?
done
echo done
