"""Per-tile SQ counters of the decode kernel from tools/pmc_ablate.sh output."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_ablate"
tiles = int(sys.argv[2]) if len(sys.argv) > 2 else (1 << 24) // 64
for d in sorted(glob.glob(os.path.join(root, "*"))):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    acc = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if "decode_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    row = {k: sum(v) / len(v) for k, v in acc.items()}
    print(os.path.basename(d), " ".join(f"{k.replace('SQ_', '')}={row[k] / tiles:.1f}" for k in sorted(row)))
