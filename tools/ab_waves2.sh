#!/bin/bash
# A/B of a variant tree (arg 1) against the working tree on config 2 at the default 4 and at 2
# waves per SIMD, alternating twice on one box.  usage: bash tools/ab_waves2.sh ab_eN [config]
V=$1; C=${2:-udp64}
mkdir -p gpurun_out/ab
run() { tag=$1; dir=$2; shift 2; (cd $dir && timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 50 "$@") > gpurun_out/ab/$tag.log 2>&1; python -c "import json; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)"; }
for k in 1 2; do
  run ${C}_base_w4_$k . --config $C
  run ${C}_var_w4_$k $V --config $C
  run ${C}_base_w2_$k . --config $C --tune waves_per_simd=2
  run ${C}_var_w2_$k $V --config $C --tune waves_per_simd=2
done
