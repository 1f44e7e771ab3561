# A/B of the LDS window size for the register-staged kernel (diagnostic; same box, one call)
set -e
mkdir -p gpurun_out/ab
run() { tag=$1; shift; timeout -k 10 120 "$@" > gpurun_out/ab/$tag.log 2>&1; python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for c in ${@:-udp64 imix}; do
  for w in 4096 8192; do
    run ${c}_full_w$w python bench.py --no-cpu-baseline --steps 50 --config $c --tune window_bytes=$w
    run ${c}_skel_w$w python bench.py --no-cpu-baseline --steps 50 --config $c --tune window_bytes=$w --ablate nodecode
  done
done
