#!/bin/bash
# A/B of the drop-in replay (scripts/dropin_probe.py) between the library in
# lachesis-base_amd/build (A) and a second build in lachesis-base_amd/build_ab
# (B), alternated on one box: A B A B.
cd "$(dirname "$0")/../.."
O=${OUT:-gpurun_out/fcc_ab}
mkdir -p $O
L=lachesis-base_amd/build/liblachesis_hip.so
cp $L $O/a.so || exit 1
for i in 1 2; do
  cp $O/a.so $L && timeout -k 10 200 python3 scripts/dropin_probe.py > $O/a_$i.json 2> $O/a_$i.err || { cp $O/a.so $L; exit 1; }
  cp ${BLIB:-lachesis-base_amd/build_ab/liblachesis_hip.so} $L && timeout -k 10 200 python3 scripts/dropin_probe.py > $O/b_$i.json 2> $O/b_$i.err || { cp $O/a.so $L; exit 1; }
done
cp $O/a.so $L
rm -f $O/a.so
for f in $O/a_1 $O/b_1 $O/a_2 $O/b_2; do python3 -c "
import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['events_per_sec']), round(d['index_seconds']*1e3,1), round(d['caller_seconds']*1e3,1))"; done
