#!/bin/bash
# rocprofv3 evidence for one bench config: kernel trace + stats, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ instruction/wait counters).  Output: gpurun_out/prof/<cfg>/
# usage: tools/prof_round.sh CFG [STEPS]
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
CFG=$1
STEPS=${2:-20}
D=gpurun_out/prof/$CFG
mkdir -p "$D"
B="python3 bench.py --config $CFG --steps $STEPS --warmup 3 --lean ${EXTRA:-}"
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" --output-format csv -d "$D/$name" -o "$name" -- $B > "$D/$name.log" 2>&1
  local rc=$?
  echo "$CFG $name rc=$rc"
  return $rc
}
run kt --kernel-trace --stats &&
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE &&
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
# clock and occupancy: effective shader clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time
# (MI355X_MICROARCH.md "DVFS give-back"); SQ_WAVE_CYCLES (quad-cycles) over it: resident waves per CU
run clk --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES
# optional LDS pass (PROF_LDS=1): bank conflicts and LDS-array cycles of the decode kernel
if [ "${PROF_LDS:-0}" = 1 ]; then
  run lds --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES
fi
