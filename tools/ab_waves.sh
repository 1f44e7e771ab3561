# A/B of the fast kernel's resident waves per SIMD (gpd_tuning.waves_per_simd), same box.
# usage: bash tools/ab_waves.sh "udp64 vxlan" "2 3 4"
set -e
mkdir -p gpurun_out/ab
for c in ${1:-udp64}; do
  for k in 1 2; do
    for w in ${2:-2 3 4}; do
      tag=${c}_w${w}_$k
      timeout -k 10 150 python bench.py --no-cpu-baseline --steps 50 --config $c --tune waves_per_simd=$w > gpurun_out/ab/$tag.log 2>&1
      python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done
