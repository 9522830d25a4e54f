#!/usr/bin/env python3
"""Summarises a tools/gpu_prof.sh output directory (rocprofv3 CSVs) into profiles/<tag>_<workload>.json + .md.

HBM traffic follows /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are kilobytes; on gfx950
FETCH_SIZE reads half of a wide coalesced stream, so the read side is doubled; WRITE_SIZE is exact for 16-B stores.
"""
import csv
import collections
import json
import os
import re
import sys


KERNELS = ("gcm_batch_kernel", "gcm_chunked_kernel")


def load(path):
    return list(csv.DictReader(open(path))) if os.path.exists(path) else []


def main(src, dst_prefix, records=None):
    stats = {}
    for r in load(os.path.join(src, "trace_kernel_stats.csv")):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                            "max_ns": float(r["MaxNs"]), "pct": float(r["Percentage"])}
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2"):
        for r in load(os.path.join(src, f + "_counter_collection.csv")):
            if any(k in r["Kernel_Name"] for k in KERNELS):
                counters[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"source": src, "records": records, "kernels": {}}
    for name, st in stats.items():
        if not any(k in name for k in KERNELS) and "keyset" not in name:
            continue
        k = {"trace": st}
        c = {n: sum(v) / len(v) for n, v in counters.get(name, {}).items()}
        if c:
            k["counters_avg_per_dispatch"] = c
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                k["hbm_read_bytes_corrected"] = c["FETCH_SIZE"] * 1024 * 2
                k["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
                k["hbm_bytes_per_launch"] = k["hbm_read_bytes_corrected"] + k["hbm_write_bytes"]
            if "GRBM_GUI_ACTIVE" in c:
                k["effective_clock_GHz"] = c["GRBM_GUI_ACTIVE"] / 8 / (st["avg_ns"])
        out["kernels"][name] = k
    # the seal instantiations gcm_*_kernel<NR, false[, ...]> of one launch: since round 4 a launch may be the W8 pair
    # (EXT 0 and EXT 3 kernels, one dispatch each), so the per-launch bytes are the sum over the seal (open) kernels
    for side, pat in (("seal", r"<\d+, false[,>]"), ("open", r"<\d+, true[,>]")):
        ks = [v for n, v in out["kernels"].items() if re.search(pat, n) and "hbm_bytes_per_launch" in v]
        if ks:
            out[f"{side}_hbm_read_bytes"] = sum(v["hbm_read_bytes_corrected"] for v in ks)
            out[f"{side}_hbm_write_bytes"] = sum(v["hbm_write_bytes"] for v in ks)
            out[f"{side}_hbm_bytes_per_launch"] = out[f"{side}_hbm_read_bytes"] + out[f"{side}_hbm_write_bytes"]
            out[f"{side}_kernel_ms_per_launch"] = sum(v["trace"]["avg_ns"] for v in ks) / 1e6
    json.dump(out, open(dst_prefix + ".json", "w"), indent=1)
    with open(dst_prefix + ".md", "w") as f:
        f.write(f"# rocprofv3 summary: {os.path.basename(dst_prefix)}\n\nsource: `{src}`\n\n")
        f.write("| kernel | calls | avg ms | min ms | HBM read (corr.) GB | HBM write GB | clock GHz |\n|---|---|---|---|---|---|---|\n")
        for n, k in out["kernels"].items():
            t = k["trace"]
            f.write(f"| `{n[:60]}` | {t['calls']} | {t['avg_ns'] / 1e6:.3f} | {t['min_ns'] / 1e6:.3f} | "
                    f"{k.get('hbm_read_bytes_corrected', 0) / 1e9:.3f} | {k.get('hbm_write_bytes', 0) / 1e9:.3f} | "
                    f"{k.get('effective_clock_GHz', 0):.2f} |\n")
        for n, k in out["kernels"].items():
            if "counters_avg_per_dispatch" in k:
                f.write(f"\n`{n}` counters (avg per dispatch):\n\n")
                for cn, cv in sorted(k["counters_avg_per_dispatch"].items()):
                    f.write(f"- {cn}: {cv:.4g}\n")
    print("wrote", dst_prefix + ".json/.md")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None)
