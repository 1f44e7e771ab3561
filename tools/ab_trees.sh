# A/B/C: bench the same configs from several trees (each a full checkout with its own built
# libgpd.so: ab_old/, ab_v1/, ... and . for the working tree), alternating on one box.
# usage: bash tools/ab_trees.sh "udp64 vxlan" ab_old ab_v1 .
set -e
mkdir -p gpurun_out/ab
cfgs=$1; shift
for c in $cfgs; do
  for k in 1 2; do
    for t in "$@"; do
      tag=${c}_$(basename $(realpath $t))$k
      (cd $t && timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 50 --config $c) > gpurun_out/ab/$tag.log 2>&1
      python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done
