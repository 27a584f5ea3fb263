#!/bin/bash
# Round 6: walk time against the L2's memory-side write requests, dispatch by
# dispatch: NP processes of scripts/probes/walk_modes2.py (two fresh handles x
# three walks each) under one rocprofv3 PMC pass each (TCC_EA0_WRREQ,
# _WRREQ_64B, _WRREQ_STALL, _RDREQ); the kernel's duration comes from the same
# CSV.  Does a slow walk write more requests?
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r06_mpmc}
mkdir -p $O
L=${LIB:-build}
for i in $(seq 1 ${NP:-6}); do
  LX_LIB=lachesis-base_amd/$L/liblachesis_hip.so WM_INST=2 WM_WALKS=3 timeout -s KILL 180 \
    rocprofv3 --kernel-include-regex k_index --output-format csv \
    --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_WRREQ_STALL TCC_EA0_RDREQ -d $O/p$i -o p \
    -- python3 scripts/probes/walk_modes2.py > $O/p$i.log 2>&1 || exit $?
done
echo done
