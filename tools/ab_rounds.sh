set -e
mkdir -p gpurun_out/ab
for c in ${CONFIGS:-vxlan imix mixed}; do
  for k in 1 2 3; do
    for d in . ab_e4096 ab_e16384; do
      tag=${c}_$(basename $d)_$k
      (cd $d && timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 50 --config $c) > gpurun_out/ab/$tag.log 2>&1
      python -c "import json; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], flush=True)"
    done
  done
done
