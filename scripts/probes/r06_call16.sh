set -o pipefail
# Per walk: the time KFD kept this process's queues evicted (and its page
# moves) -- several walk processes in a row
O=gpurun_out/r06_evict
mkdir -p $O
for i in 1 2 3 4 5; do
  WM_INST=1 WM_WALKS=5 timeout -k 10 200 python3 scripts/probes/walk_modes2.py >> $O/walks.jsonl 2>> $O/walks.err || exit $?
done
cat $O/walks.jsonl
