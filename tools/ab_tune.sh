#!/bin/bash
# A/B on one GPU box over trees and --tune settings, alternating, two rounds:
# usage: tools/ab_tune.sh "dir[:tune] dir[:tune] ..." config [config ...]
set -e
mkdir -p gpurun_out/ab
VARS=$1; shift
for c in "$@"; do
  for k in 1 2; do
    for v in $VARS; do
      d=${v%%:*}; t=${v#*:}; [ "$t" = "$v" ] && t=""
      tag=${c}_$(basename $d)${t:+_$t}_$k
      (cd $d && timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 50 --config $c ${t:+--tune $t}) > gpurun_out/ab/$tag.log 2>&1
      python -c "import json; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], flush=True)"
    done
  done
done
