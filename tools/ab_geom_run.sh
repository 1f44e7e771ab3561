#!/bin/bash
# round 6: fallback lists decoded per workgroup — full GPU suite, then same-box A/B against ab_old
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_wg.log 2>&1 || { tail -40 gpurun_out/gputest_wg.log; exit 1; }
tail -1 gpurun_out/gputest_wg.log
bash tools/ab_tune.sh "ab_old . ab_old:grid_rounds=8 .:grid_rounds=8" mixed imix udp64 2>&1 | tee gpurun_out/ab_wgfb.txt
