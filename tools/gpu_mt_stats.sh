# combining statistics of the per-record path at 1, 4 and 16 threads, 1200-byte records, combine 0 / 1 / 2 / 4
set +e
cd $GRAFT_REPO_ROOT
for C in 0 1 2 4; do
  for T in 1 4 16; do
    PTLS_MI355X_COMBINE_STATS=1 PTLS_MI355X_COMBINE=$C MT_THREADS=$T timeout -k 10 60 tools/_bin/mt_records 0.5 1200 > gpurun_out/mts.log 2>&1; rc=$?
    echo "== combine=$C threads=$T rc=$rc"; grep -v amdgpu.ids gpurun_out/mts.log | grep -E "threads +$T:|combine stats"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
