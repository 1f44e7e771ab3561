# A/B of launch geometry knobs for the register-staged kernel (diagnostic; same box, one call)
set -e
mkdir -p gpurun_out/ab
run() { tag=$1; shift; timeout -k 10 120 env "$@" > gpurun_out/ab/$tag.log 2>&1; python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for w in 4 2 3; do
  run full_w$w GPD_RS_MINW=$w python bench.py --no-cpu-baseline --steps 50
  run skel_w$w GPD_RS_MINW=$w python bench.py --no-cpu-baseline --steps 50 --ablate nodecode
done
