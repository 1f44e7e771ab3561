set -e
mkdir -p gpurun_out
for k in 1 2; do
for v in "." "ab_e8"; do
  (cd $v && timeout -k 10 150 python bench.py --config mixed --lean --no-cpu-baseline --steps 50) > gpurun_out/m_$(basename $v)_$k.log 2>&1
  tail -1 gpurun_out/m_$(basename $v)_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
timeout -k 10 150 python bench.py --config mixed --lean --no-cpu-baseline --steps 50 --decoders novxlan > gpurun_out/m_novx_$k.log 2>&1
tail -1 gpurun_out/m_novx_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('novxlan', d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 150 python bench.py --config mixed --lean --no-cpu-baseline --steps 50 --tune header_once=0 > gpurun_out/m_ho0_$k.log 2>&1
tail -1 gpurun_out/m_ho0_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ho0', d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 150 python bench.py --config mixed --lean --no-cpu-baseline --steps 50 --ablate nodecode > gpurun_out/m_skel_$k.log 2>&1
tail -1 gpurun_out/m_skel_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('skeleton', d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
