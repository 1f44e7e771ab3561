# A/B: a previous build of the whole tree (ab_old/: a checkout of an earlier commit with its own
# libgpd.so, made by `git worktree add ab_old <rev> && (cd ab_old && python -m gopacket_amd.build)`)
# vs the working tree, alternating on the same box.  usage: bash tools/ab_lib.sh [configs...]
set -e
mkdir -p gpurun_out/ab
run() { tag=$1; dir=$2; shift 2; (cd $dir && timeout -k 10 150 "$@") > gpurun_out/ab/$tag.log 2>&1; python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for c in ${@:-udp64 pcap64}; do
  for k in 1 2; do
    run ${c}_prev$k ab_old python bench.py --no-cpu-baseline --lean --steps 50 --config $c
    run ${c}_new$k . python bench.py --no-cpu-baseline --lean --steps 50 --config $c
  done
done
