set -o pipefail
# KFD's per-process view while a walk process runs: queues and CU occupancy
# of every process holding the GPU (ours and others')
O=gpurun_out/r06_kfd
mkdir -p $O
WM_INST=2 WM_WALKS=4 timeout -k 10 200 python3 scripts/probes/walk_modes2.py > $O/walks.jsonl 2> $O/walks.err &
P=$!
for i in 1 2 3 4 5 6 7 8; do
  sleep 2
  {
    echo "== sample $i $(date +%s.%N)"
    for d in /sys/class/kfd/kfd/proc/*; do
      [ -d "$d" ] || continue
      echo "pid $(basename $d)"
      for f in $(find $d -maxdepth 3 -type f 2>/dev/null | head -60); do
        v=$(timeout 2 head -c 200 $f 2>/dev/null | tr '\n' ' ')
        echo "  ${f#$d/} = $v"
      done
    done
  } >> $O/kfd_proc.txt 2>&1
done
wait $P; rc=$?
cat $O/walks.jsonl
exit $rc
