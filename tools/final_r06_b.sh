#!/bin/bash
# round 6 final evidence, part B: profiles of configs 3 (IMIX), 5 (pcap64) and the traffic mix
cd "${GRAFT_REPO_ROOT:-.}"
rm -rf gpurun_out/prof
tools/prof_round.sh imix 20 && tools/prof_round.sh pcap64 20 && tools/prof_round.sh mixed 20
