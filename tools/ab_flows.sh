#!/bin/bash
# A/B of the F3 flow insert on one box: trees (each with its own built libgpd.so; default
# ab_old/ against the working tree), alternating, two rounds; prints insert_ms (new flows),
# existing_flows.insert_ms and bursts16.insert_ms.
# usage: bash tools/ab_flows.sh [DIR ...]
set -e
mkdir -p gpurun_out/ab
[ $# -gt 0 ] || set -- ab_old .
run() { tag=$1; dir=$2; (cd $dir && timeout -k 10 200 python bench.py --no-cpu-baseline --lean --steps 10 --flows) > gpurun_out/ab/$tag.log 2>&1; python -c "
import json
for l in open('gpurun_out/ab/$tag.log'):
    if l.startswith('{') and 'existing_flows' in l:
        d = json.loads(l); b = d.get('bursts16', {})
        print('$tag', d['insert_ms'], d['existing_flows']['insert_ms'], b.get('insert_ms', b), flush=True)"; }
for k in 1 2; do
  for t in "$@"; do run flows_$(basename $(realpath $t))$k $t; done
done
