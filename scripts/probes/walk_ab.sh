#!/bin/bash
# A/B of a walker change: scripts/probes/walk_time.py alternately on the
# baseline build (make ab: the change compiled out by -DLX_AB_BASE) and the
# shipped build, R rounds each, one JSON line per run.
#   OUT=gpurun_out/wab R=3 bash scripts/probes/walk_ab.sh     (WT_V / WT_EPV / WT_OPTS pass through)
#   AB_OPTS='{"crec": 0}' ...: the shipped build with those options against its defaults
cd "$(dirname "$0")/../.."
O=${OUT:-gpurun_out/wab}
mkdir -p $O
for i in $(seq 1 ${R:-3}); do
  # SWAP=1: the shipped build first in each pair
  L1=${LIB_A:-lachesis-base_amd/build_ab/liblachesis_hip.so} L2=${LIB_B:-lachesis-base_amd/build/liblachesis_hip.so}
  [ "${SWAP:-0}" = 1 ] && { t=$L1; L1=$L2; L2=$t; }
  if [ -n "$AB_OPTS" ]; then
    # one library, an option set A/B instead: WT_OPTS=$AB_OPTS against the default
    WT_OPTS="$AB_OPTS" timeout -k 10 240 python3 scripts/probes/walk_time.py >> $O/walk_ab.jsonl || exit $?
    timeout -k 10 240 python3 scripts/probes/walk_time.py >> $O/walk_ab.jsonl || exit $?
    continue
  fi
  for lib in $L1 $L2; do
    LX_LIB=$lib timeout -k 10 240 python3 scripts/probes/walk_time.py >> $O/walk_ab.jsonl || exit $?
  done
done
cat $O/walk_ab.jsonl
