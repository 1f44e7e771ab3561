#!/bin/bash
# SQ instruction/wait counters of the decode kernel per ablation (diagnostics), gpurun_out/pmc_ablate/
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/pmc_ablate
mkdir -p $D
CFG="${CFG:-udp64}"
for ab in full ${ABLATIONS:-nocsum,nohash nodecode}; do
  extra=""
  [ "$ab" != full ] && extra="--ablate $ab"
  name=${ab//,/_}
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --output-format csv -d $D/$name -o $name -- python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline $extra > $D/$name.log 2>&1
  rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
