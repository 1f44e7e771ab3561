#!/bin/bash
# A/B/C... on one GPU box: bench.py from several trees (each with its own libgpd.so), alternating,
# two rounds.  usage: tools/ab_dirs.sh "dir1 dir2 ..." config [config ...]
set -e
mkdir -p gpurun_out/ab
DIRS=$1; shift
run() { tag=$1; dir=$2; shift 2; (cd $dir && timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 50 "$@") > gpurun_out/ab/$tag.log 2>&1; python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], flush=True)"; }
for c in "$@"; do
  for k in 1 2; do
    for d in $DIRS; do run ${c}_$(basename $d)_$k $d --config $c; done
  done
done
