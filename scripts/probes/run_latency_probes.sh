#!/bin/bash
# Host-wait latency probe and drop-in replays at several FC cache sizes.
cd "$(dirname "$0")/../.."
O=${OUT:-gpurun_out/latprobe}
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -Wno-unused-value -Wno-unused-result -o $O/sync_latency scripts/probes/sync_latency.hip || exit $?
timeout -k 10 60 $O/sync_latency > $O/sync_latency.json 2>&1 || exit $?
for W in ${FCC:-1024 2048 4032}; do
  timeout -k 10 200 python3 scripts/dropin_probe.py --fc-cache $W > $O/dropin_$W.json 2> $O/dropin_$W.err || exit $?
done
echo done
