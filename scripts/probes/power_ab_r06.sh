#!/bin/bash
# Round 6: the walk's power against its clock.  For each library in LIBS, one
# process walks C3 WM_WALKS times back to back (scripts/probes/walk_modes2.py,
# the shipped walk-clock record per walk) while amd-smi samples the socket
# power and the GFX clocks (read-only); power_ab.py pairs the samples that fall
# inside the walks with the walks' clocks and cycles.
cd "$(dirname "$0")/../.."
O=${OUT:-gpurun_out/r06_power}
mkdir -p $O
timeout -k 5 60 amd-smi static --limit --json > $O/limit.json 2>&1 || true
for L in ${LIBS:-build build_pNOLA build_pNOHB}; do
  ( while true; do echo "T $(date +%s.%N)"; timeout -k 2 10 amd-smi metric -p -c --json 2>/dev/null; sleep 0.2; done ) > $O/trace_$L.txt 2>&1 &
  SAMP=$!
  LX_LIB=lachesis-base_amd/$L/liblachesis_hip.so WM_INST=1 WM_WALKS=${WM_WALKS:-80} WM_SHIPCLK=1 \
    timeout -k 10 300 python3 scripts/probes/walk_modes2.py > $O/walks_$L.jsonl 2> $O/walks_$L.err
  rc=$?
  kill $SAMP 2>/dev/null; wait $SAMP 2>/dev/null
  [ $rc = 0 ] || exit $rc
  sleep ${COOL:-5}
done
echo done
