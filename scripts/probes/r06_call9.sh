set -o pipefail
mkdir -p gpurun_out/r06_recpf
# record prefetch A/B, settings interleaved walk by walk in each process
for i in 1 2 3; do
  WL_OPT=rec_pf WL_VALUES=0,24,64,160 WL_ROUNDS=3 timeout -k 10 300 python3 scripts/probes/walk_lock_ab.py >> gpurun_out/r06_recpf/recpf_ab.jsonl 2>> gpurun_out/r06_recpf/recpf_ab.err || exit $?
done

AB_ROUNDS=4 timeout -k 10 300 python3 scripts/probes/abft_rfc_ab.py > gpurun_out/r06_recpf/abft_rfc_ab.jsonl 2> gpurun_out/r06_recpf/abft_rfc_ab.err || exit $?
cat gpurun_out/r06_recpf/abft_rfc_ab.jsonl
