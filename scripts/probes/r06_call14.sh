set -o pipefail
# Which processes hold the GPU while a walk process runs (the slow mode's
# group-wise stall quanta look like preemption by another queue's work)?
O=gpurun_out/r06_procs
mkdir -p $O
WM_INST=2 WM_WALKS=4 timeout -k 10 200 python3 scripts/probes/walk_modes2.py > $O/walks.jsonl 2> $O/walks.err &
P=$!
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  sleep 2
  timeout -k 5 20 amd-smi process --json > $O/proc_$i.json 2>&1
  timeout -k 5 20 rocm-smi --showpids > $O/pids_$i.txt 2>&1
done
wait $P; rc=$?
cat $O/walks.jsonl
ls /proc | grep -E '^[0-9]+$' | while read p; do [ -r /proc/$p/cmdline ] && echo "$p $(tr '\0' ' ' < /proc/$p/cmdline | cut -c1-150)"; done > $O/ps.txt 2>/dev/null
exit $rc
