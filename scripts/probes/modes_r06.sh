#!/bin/bash
# Round 6: the walk's two modes.  (1) WM processes of scripts/probes/walk_modes2.py
# per library (shipped build, LowestAfter stores off, HB stores off), two fresh
# Index handles per process: does the mode follow the process, the allocation,
# or the stores?  (2) one PMC pass per library of the L2's memory-side write and
# read request counters (plus their stall / level counters where this
# rocprofv3 lists them) over one walk process.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r06_modes}
mkdir -p $O
LIBS=${LIBS:-"build build_pNOLA build_pNOHB"}
for i in $(seq 1 ${WM:-3}); do
  for L in $LIBS; do
    LX_LIB=lachesis-base_amd/$L/liblachesis_hip.so WM_INST=${WM_INST:-2} WM_WALKS=3 \
      timeout -k 10 240 python3 scripts/probes/walk_modes2.py >> $O/modes.jsonl || exit $?
  done
done
[ "${PMC:-1}" = 1 ] || exit 0
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
have() { grep -q "\b$1\b" $O/avail.txt; }
PA="TCC_EA0_WRREQ TCC_EA0_WRREQ_64B"
for c in TCC_EA0_WRREQ_STALL TCC_EA0_WRREQ_LEVEL; do have $c && PA="$PA $c"; done
PB="TCC_EA0_RDREQ"
for c in TCC_EA0_RDREQ_LEVEL TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ_DRAM; do have $c && PB="$PB $c"; done
for L in $LIBS; do
  for P in A B; do
    eval C=\$P$P
    LX_LIB=lachesis-base_amd/$L/liblachesis_hip.so WM_INST=1 WM_WALKS=2 timeout -s KILL 180 \
      rocprofv3 --kernel-include-regex k_index --output-format csv --pmc $C -d $O/pmc_${L}_$P -o p \
      -- python3 scripts/probes/walk_modes2.py > $O/pmc_${L}_$P.log 2>&1 || exit $?
  done
done
echo done
