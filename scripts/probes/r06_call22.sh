set -o pipefail
O=gpurun_out/r06_fcdepth
mkdir -p $O
timeout -k 10 300 python3 scripts/probes/fc_depth_ab.py > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.json
