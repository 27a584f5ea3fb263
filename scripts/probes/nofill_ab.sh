#!/bin/bash
# Fill-off A/B of the shipped C3 walk: the default build and the timing-only
# build without the LowestAfter range fill (make nofill), alternated A B A B
# on the same box.  OUT=gpurun_out/nofill bash scripts/probes/nofill_ab.sh
cd "$(dirname "$0")/../.."
O=${OUT:-gpurun_out/nofill}
mkdir -p $O
: > $O/ab.jsonl
for k in 1 2; do
  timeout -k 10 200 python3 scripts/probes/walk_time.py >> $O/ab.jsonl 2> $O/a$k.err || exit $?
  LX_LIB=$PWD/lachesis-base_amd/build_nofill/liblachesis_hip.so timeout -k 10 200 python3 scripts/probes/walk_time.py >> $O/ab.jsonl 2> $O/b$k.err || exit $?
done
cat $O/ab.jsonl
