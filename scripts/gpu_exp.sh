#!/bin/bash
# Experiment session: parity tests, then benches (each step time-limited;
# stop on a fault/timeout).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 5 "gpurun_out/$name.log" | cut -c1-1500
  if [ $rc -gt 1 ]; then exit $rc; fi
  return 0
}
for spec in "$@"; do
  eval "$spec"
done
