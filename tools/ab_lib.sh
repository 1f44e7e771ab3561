# A/B: the committed library (tools/ab_libgpd_prev.so, built from HEAD) vs the working tree's,
# alternating on the same box.  usage: bash tools/ab_lib.sh [configs...]
set -e
mkdir -p gpurun_out/ab
run() { tag=$1; shift; timeout -k 10 150 env "$@" > gpurun_out/ab/$tag.log 2>&1; python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for c in ${@:-udp64 pcap64}; do
  for k in 1 2; do
    run ${c}_prev$k GPD_LIB_PATH=tools/ab_libgpd_prev.so python bench.py --no-cpu-baseline --steps 50 --config $c
    run ${c}_new$k python bench.py --no-cpu-baseline --steps 50 --config $c
  done
done
