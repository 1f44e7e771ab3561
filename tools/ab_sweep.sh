#!/bin/bash
# Tuning sweep on one box (gpd_ctx_set_tuning through bench.py --tune): each config at its
# default and at other window sizes / waves per SIMD, alternating twice.  usage: bash tools/ab_sweep.sh
mkdir -p gpurun_out/sweep
run() { tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 50 "$@" > gpurun_out/sweep/$tag.log 2>&1; python -c "import json; d=json.loads(open('gpurun_out/sweep/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)"; }
for k in 1 2; do
  run udp64_def$k --config udp64
  run udp64_w8k2$k --config udp64 --tune window_bytes=8192,waves_per_simd=2
  run udp64_w8k3$k --config udp64 --tune window_bytes=8192,waves_per_simd=3
  run udp64_w4k2$k --config udp64 --tune window_bytes=4096,waves_per_simd=2
  run udp64_w4k3$k --config udp64 --tune window_bytes=4096,waves_per_simd=3
  run vxlan_def$k --config vxlan
  run vxlan_w2$k --config vxlan --tune waves_per_simd=2
  run imix_def$k --config imix
  run imix_w2$k --config imix --tune waves_per_simd=2
done
