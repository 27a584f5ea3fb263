set -o pipefail
O=gpurun_out/r06_fc16
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_abft.py tests/test_gpu_fccache.py tests/test_gpu_dropin.py > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 scripts/probes/abft_fc16_ab.py > $O/fc16_ab.jsonl 2> $O/fc16_ab.err || exit $?
cat $O/fc16_ab.jsonl
AB_OPT=claimed_batch timeout -k 10 300 python3 scripts/probes/abft_fc16_ab.py > $O/claimed_batch_ab.jsonl 2> $O/claimed_batch_ab.err || exit $?
cat $O/claimed_batch_ab.jsonl
AB_OPT=elect_ahead AB_VALUES=2,0 timeout -k 10 300 python3 scripts/probes/abft_fc16_ab.py > $O/elect_ahead_ab.jsonl 2> $O/elect_ahead_ab.err || exit $?
cat $O/elect_ahead_ab.jsonl
timeout -k 10 300 python3 scripts/bench_abft_only.py 5 > $O/abft_leg.json 2> $O/abft_leg.err || exit $?
cat $O/abft_leg.json
