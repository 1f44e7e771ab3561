#!/bin/bash
# A/B on one GPU box: the working tree (.) against variant trees ab_e<N>/ (tools/ab_exp_build.sh),
# alternating, two rounds; prints ms_per_step and kernel_ms per run.
# usage: tools/ab_exp.sh "N1 N2" config [config ...]
set -e
mkdir -p gpurun_out/ab
VARS=$1; shift
run() { tag=$1; dir=$2; shift 2; (cd $dir && timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 50 "$@") > gpurun_out/ab/$tag.log 2>&1; python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)"; }
for c in "$@"; do
  for k in 1 2; do
    run ${c}_base$k . --config $c
    for N in $VARS; do run ${c}_e${N}_$k ab_e$N --config $c; done
  done
done
