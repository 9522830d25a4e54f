#!/usr/bin/env python3
"""Summarises rocprofv3 --pmc runs of tools/ct_probe*.py: per kernel, the SQ_LDS_BANK_CONFLICT and SQ_INSTS_LDS values
of every dispatch, one line per (case) directory, so that equal shapes under different keys and payloads can be
compared.

    python tools/ct_summary.py gpurun_out/ctpr > profiles/r3_ct_perrec.txt
"""
import collections
import csv
import glob
import os
import sys


def main(root):
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for f in files:
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if "gcm_" not in name and "span" not in name:
                    continue
                short = name.split("(")[0].replace("void ", "")
                vals[short][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        print(os.path.basename(d))
        for k in sorted(vals):
            c = {n: [int(v) for _, v in sorted(x)] for n, x in vals[k].items()}
            print(f"  {k:42s} conflicts {c.get('SQ_LDS_BANK_CONFLICT')}  lds insts {c.get('SQ_INSTS_LDS')}")


if __name__ == "__main__":
    main(sys.argv[1])
