set -o pipefail
mkdir -p gpurun_out/r06_skew
LX_LIB=lachesis-base_amd/build_pSKEW/liblachesis_hip.so timeout -k 10 240 python3 scripts/probes/walk_skew.py > gpurun_out/r06_skew/skew.jsonl 2> gpurun_out/r06_skew/skew.err || exit $?
cat gpurun_out/r06_skew/skew.jsonl
OUT=gpurun_out/r06_reh GS=2 T=500 bash scripts/rowseg_rehearsal.sh
