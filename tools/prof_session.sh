#!/bin/bash
# rocprofv3 passes over the decode kernel (kernel trace + separate PMC passes), outputs under gpurun_out/prof
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
CFG="${1:-udp64}"
TAG="${2:-r01}"
B="python3 bench.py --config $CFG --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline"
D=gpurun_out/prof_${TAG}_${CFG}
mkdir -p $D
rocprofv3 -L > $D/counters_list.txt 2>&1 || true
run() { # name, extra args
  local name=$1; shift
  echo "== $name"
  timeout -k 10 400 rocprofv3 "$@" --output-format csv -d $D/$name -o $name -- $B > $D/$name.log 2>&1
  local rc=$?
  echo "rc=$rc"; tail -2 $D/$name.log
  [ $rc -eq 0 ] || exit $rc
}
run kt --kernel-trace --stats
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
