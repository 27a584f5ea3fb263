#!/bin/bash
# One GPU session: build check, parity tests, smoke, short bench.
# Each GPU step has its own time limit; a fault/timeout (rc >= 124 or signal)
# stops the script, ordinary test failures (rc 1) do not stop the bench.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  return $rc
}
ok_or_fail() { [ "$1" -le 1 ]; }
step pytest_gpu ${PYTEST_T:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS}; rc=$?
ok_or_fail $rc || exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?
ok_or_fail $rc || exit $rc
step bench ${BENCH_T:-600} python bench.py ${BENCH_ARGS}; rc=$?
exit $rc
