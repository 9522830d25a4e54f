#!/bin/bash
# HBM bytes (FETCH_SIZE, WRITE_SIZE: one --pmc pass each) of engine variants tools/gv/<name> on one workload, through
# tools/ab.py (one round):  bash tools/gpu_pmc_variants.sh "<names>" <workload> <records> <tag>
set +e
names=$1; W=$2; N=$3; TAG=$4
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for v in $names; do for c in FETCH_SIZE WRITE_SIZE; do
  OUT=$R/gpurun_out/${TAG}_${v}_$c
  timeout -k 10 180 rocprofv3 --pmc $c --output-format csv -d $OUT -o p -- python3 $R/tools/ab.py $R/tools/gv/$v/libptls_mi355x.so \
      --workload $W --records $N --rounds 1 --reps 1 > $OUT.log 2>&1
  rc=$?; echo "$v $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done; done
python3 - "$R/gpurun_out" "$TAG" "$names" <<'PY'
import csv, glob, os, sys
root, tag, names = sys.argv[1], sys.argv[2], sys.argv[3].split()
for v in names:
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = []
        for f in glob.glob(os.path.join(root, f"{tag}_{v}_{c}", "**", "*counter_collection.csv"), recursive=True):
            rows += list(csv.DictReader(open(f)))
        per = {}
        for r in rows:
            if "gcm_chunked_kernel" not in r["Kernel_Name"]:
                continue
            k = (r["Kernel_Name"], r["Dispatch_Id"])
            per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
        byk = {}
        for (k, d), val in per.items():
            byk.setdefault(k, []).append(val)
        for k, vals in sorted(byk.items()):
            avg = sum(vals) / len(vals)
            gb = avg * 1024 / 1e9 * (2 if c == "FETCH_SIZE" else 1)
            print(f"{v:6s} {c:10s} {k[:60]:60s} {len(vals)} dispatches  {gb:8.3f} GB per dispatch" + (" (x2 gfx950 corr.)" if c == "FETCH_SIZE" else ""))
PY
