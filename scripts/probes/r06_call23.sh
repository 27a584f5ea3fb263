set -o pipefail
O=gpurun_out/r06_stop
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_abft.py tests/test_gpu_fccache.py tests/test_gpu_dropin.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head; exit $rc; }
AB_OPT=rfc_stop AB_VALUES=1,0 timeout -k 10 300 python3 scripts/probes/abft_fc16_ab.py > $O/stop_ab.jsonl 2> $O/stop_ab.err || exit $?
cat $O/stop_ab.jsonl
