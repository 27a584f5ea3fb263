#!/bin/bash
# Fast / slow walk modes: N walk_time.py processes in a row on the counters
# build (make wprof, copied to build_ab/liblachesis_wprof.so, which travels; LX_PROF=1 prints per-wave walker counters), one log each.
#   OUT=gpurun_out/wmodes N=4 bash scripts/probes/walk_modes.sh
cd "$(dirname "$0")/../.."
O=${OUT:-gpurun_out/wmodes}
mkdir -p $O
# AB_OPTS: odd processes run with WT_OPTS=$AB_OPTS, even ones with the defaults
for i in $(seq 1 ${N:-4}); do
  o='{}'; [ -n "$AB_OPTS" ] && [ $((i % 2)) = 1 ] && o="$AB_OPTS"
  WT_OPTS="$o" LX_PROF=1 LX_LIB=${WLIB:-lachesis-base_amd/build_ab/liblachesis_wprof.so} timeout -k 10 240 \
      python3 scripts/probes/walk_time.py > $O/p$i.log 2>&1 || exit $?
  tail -n 1 $O/p$i.log
done
