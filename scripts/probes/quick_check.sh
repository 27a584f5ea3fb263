#!/bin/bash
# Quick GPU iteration: the small-path / FC cache / drop-in tests, the level-fed
# probe and a drop-in replay (OUT=gpurun_out/quick).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/quick}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_small.py tests/test_gpu_fccache.py tests/test_gpu_dropin.py tests/test_gpu_batcher.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python3 scripts/feed_probe.py > $O/feed.json 2> $O/feed.err || exit $?
timeout -k 10 200 python3 scripts/dropin_probe.py > $O/dropin.json 2> $O/dropin.err || exit $?
echo done
