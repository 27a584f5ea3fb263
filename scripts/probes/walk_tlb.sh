#!/bin/bash
# Two walk_time.py processes back to back under the address-translation
# counters (the first process on a box walks C3 slower than the second);
# each pass a process of its own, as rocprofv3 needs.
#   OUT=gpurun_out/wtlb bash scripts/probes/walk_tlb.sh
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/wtlb}
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "TCP_UTCL1[A-Z_]*\|UTCL2[A-Z_]*\|TCP_TCP_TA_DATA_STALL[A-Z_]*\|TCP_PENDING_STALL[A-Z_]*\|TCP_WRITE_TAGCONFLICT_STALL[A-Z_]*" $O/avail.txt | sort -u > $O/names.txt || true
C="${CTRS:-TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum GRBM_GUI_ACTIVE}"
for i in 1 2 3; do
  timeout -k 10 240 rocprofv3 --kernel-include-regex k_index --output-format csv --pmc $C -d $O/p$i -o p$i -- python3 scripts/probes/walk_time.py > $O/p$i.log 2>&1 || exit $?
done
find $O -name "*trace*.csv" -delete
tail -n 1 $O/p*.log
