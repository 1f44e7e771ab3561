#!/bin/bash
# round 6 final evidence, part A: GPU suite, smoke, default bench line, profiles of configs 2 / tcp64 / 4
cd "${GRAFT_REPO_ROOT:-.}"
rm -rf gpurun_out/prof
tools/gpu_session.sh "gputest|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c \"import __graft_entry__ as g; g.smoke()\"" "bench|300|python bench.py" || exit 1
tools/prof_round.sh udp64 20 && tools/prof_round.sh tcp64 20 && PROF_LDS=1 tools/prof_round.sh vxlan 20
