#!/bin/bash
# round 6 final evidence, part C: lean vs full bench line on one box (alternating), then
# profiles of configs 2 / tcp64 with the loader/decoder split kernel
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/lf
mkdir -p gpurun_out/lf
for k in 1 2; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 50 > gpurun_out/lf/lean_$k.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/lf/full_$k.log 2>&1 || exit 1
  for f in lean full; do
    python -c "import json; d=json.loads(open('gpurun_out/lf/${f}_$k.log').read().strip().splitlines()[-1]); print('${f}_$k', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['config'].get('settle_ms'), flush=True)"
  done
done
tools/prof_round.sh udp64 20 && tools/prof_round.sh tcp64 20
