"""Attribute tools/flow_prof.py's flow-kernel launches: per rocprofv3 output dir, the
flow_insert_kernel / flow_verify_kernel dispatches in order alternate new-flow and
existing-flow inserts (reset between rounds).  Prints mean duration (kernel trace) or mean
counters (PMC csv) per (case, kernel), the first round dropped as warm-up.

    python tools/flow_prof_split.py DIR [DIR ...]
"""
import collections
import csv
import glob
import json
import sys


def rows(d):
    out = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out.append(("trace", int(r["Dispatch_Id"]), r["Kernel_Name"],
                        {"dur_us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3}))
    acc = collections.defaultdict(dict)
    names = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            acc[k][r["Counter_Name"]] = acc[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[k] = r["Kernel_Name"]
    for k, v in acc.items():
        out.append(("pmc", k, names[k], v))
    return sorted(out, key=lambda x: x[1])


def split(d):
    seq = [r for r in rows(d) if "flow_insert_kernel" in r[2] or "flow_verify_kernel" in r[2]]
    groups = collections.defaultdict(list)
    for j, (_, _, name, vals) in enumerate(seq):
        rnd, pos = divmod(j, 4)  # insert,verify (new) then insert,verify (existing)
        if rnd == 0:
            continue
        case = "new" if pos < 2 else "existing"
        kern = "insert" if "insert" in name else "verify"
        groups[(case, kern)].append(vals)
    res = {}
    for key, lst in sorted(groups.items()):
        keys = lst[0].keys()
        res[f"{key[0]}/{key[1]}"] = {k: round(sum(x[k] for x in lst) / len(lst), 3) for k in keys}
        res[f"{key[0]}/{key[1]}"]["launches"] = len(lst)
    return res


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(d)
        print(json.dumps(split(d), indent=1))
