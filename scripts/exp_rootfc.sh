cd /root/repo
mkdir -p gpurun_out/exp1
for w in 1024 2048 4096 512; do
LX_ROOTFC_WGS=$w timeout -k 10 120 python3 scripts/bench_abft_only.py 5 > gpurun_out/exp1/w$w.json 2>/dev/null || exit $?
done
export TMPDIR=/tmp
for w in 1024 2048 4096; do
LX_ROOTFC_WGS=$w timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp1/k$w -o k -- python3 scripts/bench_abft_only.py 3 > /dev/null 2>&1 || exit $?
done
find gpurun_out/exp1 -name "*trace*.csv" -delete
