#!/bin/bash
# round 6 final evidence, part D (after the packed descriptor layout): GPU suite, smoke, the
# default bench line, then profiles of configs 2 / tcp64 with the shipped sp_kernel
cd "${GRAFT_REPO_ROOT:-.}"
rm -rf gpurun_out/prof
tools/gpu_session.sh "gputest|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c \"import __graft_entry__ as g; g.smoke()\"" "bench|300|python bench.py" || exit 1
tools/prof_round.sh udp64 20 && tools/prof_round.sh tcp64 20
