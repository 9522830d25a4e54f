# per-context latency split: rocprofv3 kernel trace of tools/lat_ctx.py (setup kernel vs one-record seal vs launch costs)
set +e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/latctx -o run -- python3 $R/tools/lat_ctx.py 300 > $R/gpurun_out/latctx.log 2>&1
rc=$?; echo "rc=$rc"; grep "^{" $R/gpurun_out/latctx.log
find $R/gpurun_out/latctx -name "*kernel_stats.csv" -exec cat {} \;
exit $rc
