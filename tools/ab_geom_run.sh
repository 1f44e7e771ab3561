#!/bin/bash
# round 6: split kernel for the record form — suite, smoke, A/B, bench
set -e
export TMPDIR=/tmp
tools/gpu_session.sh "gputest|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" "smoke|120|python -c \"import __graft_entry__ as g; g.smoke()\""
grep -q " passed" gpurun_out/gputest.log && ! grep -q "failed" gpurun_out/gputest.log
bash tools/ab_tune.sh ". .:split=0" udp64 tcp64 2>&1 | tee gpurun_out/ab_split6.txt
timeout -k 10 300 python bench.py > gpurun_out/bench_split.log 2>&1
