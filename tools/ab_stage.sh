set -e
mkdir -p gpurun_out/ab
run() { tag=$1; shift; timeout -k 10 120 env "$@" > gpurun_out/ab/$tag.log 2>&1; python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for s in 4096 8192; do
  run full_$s GPD_STAGE=$s python bench.py --no-cpu-baseline --steps 50
  run skel_$s GPD_STAGE=$s python bench.py --no-cpu-baseline --steps 50 --ablate nodecode
done
run full_4096_w3 GPD_RS_MINW=3 python bench.py --no-cpu-baseline --steps 50
run full_8192_w2 GPD_STAGE=8192 GPD_RS_MINW=2 python bench.py --no-cpu-baseline --steps 50
