#!/bin/bash
# A/B of the PCIe-inclusive host path (bench.py --host MODE): the working tree (.) against ab_old/
# (a checkout of an earlier commit with its own libgpd.so), alternating, three rounds.
# usage: tools/ab_host2.sh [registered|plain] [config]
set -e
mkdir -p gpurun_out/ab
MODE=${1:-registered}; CFG=${2:-udp64}
run() { tag=$1; dir=$2; (cd $dir && timeout -k 10 200 python bench.py --no-cpu-baseline --host $MODE --steps 5 --config $CFG) > gpurun_out/ab/$tag.log 2>&1; python -c "import json; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], flush=True)"; }
for k in 1 2 3; do
  run host_${MODE}_${CFG}_prev$k ab_old
  run host_${MODE}_${CFG}_new$k .
done
