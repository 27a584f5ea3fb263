#!/bin/bash
# Round 6: the walk's shader clock (lx_last_walk_clock) over back-to-back C3
# walks, with the board's power / clocks / temperature sampled beside it
# (amd-smi metric, read-only) and its power limit (amd-smi static --limit).
cd "$(dirname "$0")/../.."
O=${OUT:-gpurun_out/r06_clkpow}
mkdir -p $O
timeout -k 5 60 amd-smi static --limit --json > $O/limit.json 2>&1 || true
timeout -k 5 60 amd-smi metric -p -c -t --json > $O/idle_metric.json 2>&1 || true
( for i in $(seq 1 200); do date +%s.%N; timeout -k 2 10 amd-smi metric -p -c -t --json 2>/dev/null; sleep 0.3; done ) > $O/metric_trace.txt 2>&1 &
SAMP=$!
WM_INST=${WM_INST:-1} WM_WALKS=${WM_WALKS:-12} WM_SHIPCLK=1 timeout -k 10 300 python3 scripts/probes/walk_modes2.py > $O/walks.jsonl 2> $O/walks.err
rc=$?
kill $SAMP 2>/dev/null
wait $SAMP 2>/dev/null
exit $rc
