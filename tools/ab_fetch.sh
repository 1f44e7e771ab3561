#!/bin/bash
# A/B of the working tree against variant trees ab_e<N>/ on one box: alternating timing runs
# (two rounds), then one FETCH_SIZE pass each (HBM read bytes per launch of the decode kernel).
# usage: tools/ab_fetch.sh "N1 N2" config
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
VARS=$1; CFG=$2
R=$PWD
mkdir -p gpurun_out/abf
tools/ab_exp.sh "$VARS" $CFG
for t in base $VARS; do
  dir=.; [ $t != base ] && dir=ab_e$t
  (cd $dir && timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/abf/$t -o fetch -- python3 bench.py --config $CFG --steps 20 --warmup 3 --lean > $R/gpurun_out/abf/$t.log 2>&1)
  python3 - $R/gpurun_out/abf/$t <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "sp_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
v = sorted(v)[len(v) // 2] if v else 0
print(sys.argv[1].split("/")[-1], "FETCH_SIZE median KB", v, "x2 bytes", 2 * 1024 * v, flush=True)
P
done
