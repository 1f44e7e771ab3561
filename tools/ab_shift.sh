# A/B: shifted (aligned network header) vs unshifted window copies, same box
set -e
mkdir -p gpurun_out/ab
run() { tag=$1; shift; timeout -k 10 150 "$@" > gpurun_out/ab/$tag.log 2>&1; python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for c in udp64 pcap64 imix vxlan; do
  run ${c}_shift python bench.py --no-cpu-baseline --steps 50 --config $c --tune shift=1
  run ${c}_noshift python bench.py --no-cpu-baseline --steps 50 --config $c --tune shift=0
done
