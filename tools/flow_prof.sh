#!/bin/bash
# F3 launch split under rocprofv3 (round 6): kernel trace, then PMC passes; gpurun_out/prof/flows/
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/prof/flows
mkdir -p $D
timeout -s KILL 60 rocprofv3 -L > $D/avail.txt 2>&1 || true
run() { local name=$1; shift; timeout -s KILL 120 rocprofv3 "$@" --output-format csv -d $D/$name -o $name -- python3 tools/flow_prof.py > $D/$name.log 2>&1; echo "flows $name rc=$?"; }
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run tcc --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum
run tcc2 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_32B_sum
