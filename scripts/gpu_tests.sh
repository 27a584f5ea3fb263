#!/bin/bash
# the whole GPU test suite (progress streams to the log), then smoke()
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/tests}
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYARGS} > $O/pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
echo done
