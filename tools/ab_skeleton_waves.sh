# Skeleton (no decode) vs full decode at 4 and 2 waves per SIMD, config 2, alternating on one box.
mkdir -p gpurun_out/skel
run() { tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 50 "$@" > gpurun_out/skel/$tag.log 2>&1; python -c "import json; d=json.loads(open('gpurun_out/skel/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)"; }
for k in 1 2; do
  run full_w4_$k --config udp64
  run skel_w4_$k --config udp64 --ablate nodecode
  run full_w2_$k --config udp64 --tune waves_per_simd=2
  run skel_w2_$k --config udp64 --tune waves_per_simd=2 --ablate nodecode
done
