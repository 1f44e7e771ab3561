"""Per-launch means of the decode kernel's PMC counters from rocprofv3 csv dirs (tools/ A/B):
    python tools/pmc_pair.py DIR [DIR ...]"""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if not any(k in r["Kernel_Name"] for k in ("rs_kernel", "ro_kernel", "decode_kernel", "sp_kernel")):
                continue
            acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    ks = list(acc.values())
    if not ks:
        print(d, "no launches")
        continue
    m = {k: sum(x[k] for x in ks) / len(ks) for k in ks[0]}
    print(d, len(ks), " ".join(f"{k}={v / 1e6:.2f}M" for k, v in sorted(m.items())))
