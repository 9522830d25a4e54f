# long per-record calls (span path): wall times, then a kernel trace of the same
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/lat_big.py 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/latbig; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o big -- python3 $GRAFT_REPO_ROOT/tools/lat_big.py > $OUT/log.txt 2>&1
rc=$?; echo rc=$rc; find $OUT -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150
exit $rc
