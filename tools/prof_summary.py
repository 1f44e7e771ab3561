"""Summarise a tools/prof_session.sh output directory (decode kernel only)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
stats = os.path.join(d, "kt", "kt_kernel_stats.csv")
for r in csv.DictReader(open(stats)):
    if "decode_kernel" in r["Name"]:
        print(f"kernel {r['Name'][:60]} calls={r['Calls']} avg={float(r['AverageNs'])/1e3:.1f}us "
              f"min={float(r['MinNs'])/1e3:.1f} max={float(r['MaxNs'])/1e3:.1f}")
agg = collections.defaultdict(list)
meta = {}
for f in glob.glob(os.path.join(d, "pmc_*", "*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "decode_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count", "SGPR_Count")}
avg = {k: sum(v) / len(v) for k, v in agg.items()}
print("dispatch:", meta)
for k in sorted(avg):
    print(f"  {k:24s} {avg[k]:16.1f}")
if "SQ_WAVES" in avg:
    w = avg["SQ_WAVES"]
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
        if k in avg:
            print(f"  {k}/wave = {avg[k]/w:.0f}")
if "SQ_WAVE_CYCLES" in avg:
    wc = avg["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        if k in avg:
            print(f"  {k}/WAVE_CYCLES = {avg[k]/wc:.3f}")
if "FETCH_SIZE" in avg:
    print(f"  HBM read (FETCH_SIZE x2 gfx950 correction) = {2*avg['FETCH_SIZE']*1024/1e9:.3f} GB/launch")
if "WRITE_SIZE" in avg:
    print(f"  HBM write (WRITE_SIZE) = {avg['WRITE_SIZE']*1024/1e9:.3f} GB/launch")
if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_ACTIVE_INST_LDS" in avg:
    print(f"  LDS bank conflict cycles / active LDS = {avg['SQ_LDS_BANK_CONFLICT']/max(1,avg['SQ_ACTIVE_INST_LDS']):.2f}")
