#!/bin/bash
# A/B of the PCIe-inclusive host path (gpd_decode_host, registered arrays) over trees,
# alternating, three rounds.  usage: bash tools/ab_host.sh "tree tree ..." [config]
set -e
mkdir -p gpurun_out/ab
cfg=${2:-udp64}
for k in 1 2 3; do
  for t in $1; do
    tag=host_${cfg}_$(basename $(realpath $t))_$k
    (cd $t && timeout -k 10 200 python bench.py --no-cpu-baseline --lean --steps 5 --config $cfg --host registered) > gpurun_out/ab/$tag.log 2>&1
    python -c "import json; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d.get('ms_per_step'), flush=True)"
  done
done
