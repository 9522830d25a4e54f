#!/usr/bin/env python3
"""Per-dispatch counter table from rocprofv3 --pmc csv output dirs: python tools/pmc_table.py <dir>... (prints, for each
dir, each kernel's counters summed over the hardware instances, per dispatch)"""
import collections
import csv
import glob
import os
import sys


def table(d):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        agg = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            agg[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (disp, cn), v in agg.items():
            out[names[disp]][cn].append(v)
    return out


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(f"== {d}")
        for k, cs in table(d).items():
            if "gcm" not in k:
                continue
            print("  " + k[:60])
            for cn, vals in sorted(cs.items()):
                print(f"    {cn:24s} " + " ".join(f"{v:.4e}" for v in vals))
