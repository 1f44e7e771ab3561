#!/bin/bash
# A/B: the default line's timed loop with HIP events around every launch vs one event pair
# around all K launches (bench.py --events), alternating on one box.  usage: bash tools/ab_events.sh
mkdir -p gpurun_out/ab
run() { tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 200 "$@" > gpurun_out/ab/$tag.log 2>&1; python -c "import json; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)"; }
for k in 1 2 3; do
  run step$k --config udp64 --events step
  run span$k --config udp64 --events span
done
