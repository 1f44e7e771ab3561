# A/B of two bench.py argument sets in the working tree, alternating on one box.
# usage: bash tools/ab_args.sh "<args A>" "<args B>" [configs...]
set -e
mkdir -p gpurun_out/ab
A=$1; B=$2; shift 2
run() { tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu-baseline --lean --steps 50 "$@" > gpurun_out/ab/$tag.log 2>&1; python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for c in ${@:-udp64 imix}; do
  for k in 1 2; do
    run ${c}_A$k --config $c $A
    run ${c}_B$k --config $c $B
  done
done
