#!/usr/bin/env python3
"""HBM traffic of the seal and open launches in a tools/gpu_prof.sh run, as multiples of the algorithmic bytes
(seal reads L + A + 40, writes L + 16; open reads L + 16 + A + 40, writes L + 1).

    python tools/traffic_ratios.py gpurun_out/prof_<tag>_<workload> <workload> <records>
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotls_amd.workloads import WORKLOADS  # noqa: E402


def ratios(summary: dict, workload: str, n: int) -> dict:
    b = WORKLOADS[workload].scaled(n).descriptors(0, n)
    L = int(b.seal["len"].astype(np.int64).sum())
    A = int(b.seal["aad_len"].astype(np.int64).sum())
    alg = {"seal": (L + A + 40 * n, L + 16 * n), "open": (L + 16 * n + A + 40 * n, L + n)}
    out = {}
    for k, (r, w) in alg.items():
        if f"{k}_hbm_read_bytes" in summary:
            out[k] = {"read": round(summary[f"{k}_hbm_read_bytes"] / r, 3), "write": round(summary[f"{k}_hbm_write_bytes"] / w, 3),
                      "total": round((summary[f"{k}_hbm_read_bytes"] + summary[f"{k}_hbm_write_bytes"]) / (r + w), 3)}
    return out


if __name__ == "__main__":
    d = json.load(open(os.path.join(sys.argv[1], "summary.json")))
    print(json.dumps(ratios(d, sys.argv[2], int(sys.argv[3]))))
