set -e
mkdir -p gpurun_out/ab
run() { tag=$1; shift; timeout -k 10 150 "$@" > gpurun_out/ab/$tag.log 2>&1; python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for c in imix vxlan udp64; do
  run ${c}_full python bench.py --no-cpu-baseline --steps 30 --config $c
  run ${c}_skel python bench.py --no-cpu-baseline --steps 30 --config $c --ablate nodecode
  run ${c}_nocsum python bench.py --no-cpu-baseline --steps 30 --config $c --ablate nocsum
done
