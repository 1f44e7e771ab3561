#!/bin/bash
# tools/prof_round.sh for one config in another tree (a variant build, tools/ab_exp_build.sh);
# its gpurun_out/prof/<cfg> is copied to gpurun_out/prof/<cfg>_<tree> here.
# usage: bash tools/prof_tree.sh TREE CFG [STEPS]
set -u
T=$1; CFG=$2; STEPS=${3:-20}
(cd "$T" && GRAFT_REPO_ROOT=. bash tools/prof_round.sh "$CFG" "$STEPS")
rc=$?
mkdir -p gpurun_out/prof
rm -rf "gpurun_out/prof/${CFG}_$(basename "$T")"
cp -r "$T/gpurun_out/prof/$CFG" "gpurun_out/prof/${CFG}_$(basename "$T")"
exit $rc
