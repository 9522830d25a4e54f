# kernel trace of per-record seals (16 B, then 1200 B): the GPU time of a lone record's launch
set +e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/latprof; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o lat -- python3 $R/tools/lat_small.py > $OUT/log.txt 2>&1
rc=$?; echo rc=$rc; find $OUT -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
g = [r for r in rows if "gcm_chunked" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in g]
import statistics
for name, part in (("16 B", d[:300]), ("1200 B", d[300:600])):
    if part:
        print(name, "median kernel us", round(statistics.median(part), 2), "n", len(part))
PY
exit $rc
