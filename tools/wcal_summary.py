#!/usr/bin/env python3
"""Summary of the tools/mb/wcal.hip calibration passes (tools/gpu_r5.sh wcal): counter bytes per dispatch ÷ the bytes
the kernel stores or loads, per access shape.   python tools/wcal_summary.py gpurun_out/wcal"""
import collections
import csv
import glob
import os
import sys


def main(src):
    for d in sorted(glob.glob(os.path.join(src, "*"))):
        name = os.path.basename(d)
        vals = collections.defaultdict(list)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if "wcal" in r["Kernel_Name"]:
                        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        log = os.path.join(src, name + ".log")
        nbytes = None
        if os.path.exists(log):
            for line in open(log):
                if "bytes" in line:
                    nbytes = int(line.rsplit("bytes", 1)[1].strip())
        for k, v in sorted(vals.items()):
            per = sorted(v)[len(v) // 2] * 1024  # KiB -> bytes, median dispatch
            ratio = per / nbytes if nbytes else float("nan")
            print(f"{name:28s} {k:11s} {per / 1e9:8.3f} GB per dispatch  ÷ bytes {ratio:6.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
