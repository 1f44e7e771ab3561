#!/bin/bash
# A/B of the TPACKET_V3 ingest (bench.py --tpv3 line) across trees, alternating, two rounds.
# usage: tools/ab_tpv3.sh "dir1 dir2 ..." [config]
set -e
mkdir -p gpurun_out/ab
DIRS=$1; CFG=${2:-udp64}
run() { tag=$1; dir=$2; (cd $dir && timeout -k 10 200 python bench.py --no-cpu-baseline --lean --steps 5 --tpv3 --config $CFG) > gpurun_out/ab/$tag.log 2>&1; python -c "
import json
for l in open('gpurun_out/ab/$tag.log'):
    l = l.strip()
    if l.startswith('{') and 'TPACKET_V3' in l:
        d = json.loads(l); print('$tag', d['Mpackets_per_s'], d['ms_per_ring'], d['GBps_ring_in'], d['walk'], flush=True)"; }
for k in 1 2; do
  for d in $DIRS; do run tpv3_${CFG}_$(basename $d)_$k $d; done
done
