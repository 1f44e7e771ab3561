#!/bin/bash
# Tile-quantization tail check: per-packet time at the default batch vs batches whose tiles are an
# exact multiple of the grid's waves (IMIX: 12,288 round-kernel waves x 5 / 6 tiles; VXLAN: 3,072 x 42 / 43).
set -e
mkdir -p gpurun_out/ab
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --lean --steps 50 "$@" > gpurun_out/ab/$tag.log 2>&1; python -c "
import json; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); n=d['config']['packets_per_gpu']; print('$tag', n, d['ms_per_step'], round(d['ms_per_step']*1e6/n,4), 'ns/pkt', d['roofline']['frac'], flush=True)"; }
for k in 1 2; do
  run imix_def_$k --config imix
  run imix_5_$k --config imix --packets 3932160
  run imix_6_$k --config imix --packets 4718592
  run vx_def_$k --config vxlan
  run vx_42_$k --config vxlan --packets 8257536
  run vx_43_$k --config vxlan --packets 8454144
done
