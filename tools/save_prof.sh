#!/bin/bash
# Copy one tools/prof_round.sh result (gpurun_out/prof/<cfg>) into profiles/<round>/<cfg>:
# summary.json (tools/prof_summary.py) + the rocprofv3 kernel stats and counter CSVs.
# usage: tools/save_prof.sh ROUND CFG [SRC_DIR]
set -eu
R=$1; CFG=$2; SRC=${3:-gpurun_out/prof/$CFG}
D=profiles/$R/$CFG
mkdir -p "$D"
python3 tools/prof_summary.py "$SRC" > "$D/summary.json"
cp "$(find "$SRC/kt" -name '*kernel_stats.csv' | head -1)" "$D/kt_kernel_stats.csv"
for p in fetch write sq lds; do
  f=$(find "$SRC/$p" -name '*counter_collection.csv' 2>/dev/null | head -1)
  [ -n "$f" ] && cp "$f" "$D/pmc_${p}_counter_collection.csv"
done
ls "$D"
