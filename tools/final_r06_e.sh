#!/bin/bash
# round 6 final evidence, part E: configs 3 / 4 / 5 and the traffic mix re-profiled with the final
# library (packed descriptors), the kernels themselves unchanged since part B
cd "${GRAFT_REPO_ROOT:-.}"
rm -rf gpurun_out/prof
tools/prof_round.sh imix 20 && PROF_LDS=1 tools/prof_round.sh vxlan 20 && tools/prof_round.sh pcap64 20 && tools/prof_round.sh mixed 20
