#!/usr/bin/env python3
"""WRITE_SIZE / FETCH_SIZE per chunked seal and open launch of each variant (tools/gpu_r5.sh wpmc), against the
workload's algorithmic bytes (bench.py's per-launch figures).   python tools/wpmc_summary.py gpurun_out/wpmc quic1200 N"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotls_amd.workloads import WORKLOADS  # noqa: E402


def main(src, workload, records):
    wl = WORKLOADS[workload].scaled(int(records))
    b = wl.descriptors(0, wl.nrecs)
    alg_w_seal = b.payload_bytes + 16 * b.n
    alg_w_open = b.payload_bytes
    for d in sorted(glob.glob(os.path.join(src, "*_*_SIZE"))):
        name, ctr = os.path.basename(d).split("_", 1)
        vals = collections.defaultdict(list)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = r["Kernel_Name"]
                    if "gcm_chunked_kernel" in k and r["Counter_Name"] == ctr:
                        vals[k].append(float(r["Counter_Value"]) * 1024)
        for k, v in sorted(vals.items()):
            big = max(v)
            if big < 1e8:
                continue
            seal = ", false," in k
            ref = (alg_w_seal if seal else alg_w_open) if ctr == "WRITE_SIZE" else None
            med = sorted(x for x in v if x > 0.5 * big)[len([x for x in v if x > 0.5 * big]) // 2]
            extra = f"  ÷ written bytes {med / ref:.3f}" if ref else ""
            print(f"{name:8s} {ctr:10s} {k[:48]:48s} {med / 1e9:7.3f} GB{extra}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
