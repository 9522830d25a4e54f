# per-record calls from T pthreads (tools/_bin/mt_records, tools/mt_build.sh) under PTLS_MI355X_COMBINE settings;
# MT_VARIANTS: engine builds (directories holding a libptls_mi355x.so) to run instead of the in-tree one
set +e
cd $GRAFT_REPO_ROOT
for V in ${MT_VARIANTS:-picotls_amd/_lib}; do
  for C in ${MT_COMBINE:-0 1 2 4}; do
    LD_LIBRARY_PATH=$V PTLS_MI355X_COMBINE=$C timeout -k 10 120 tools/_bin/mt_records ${MT_SECONDS:-0.5} ${MT_LENS:-16 1200 16384} > gpurun_out/mt.log 2>&1; rc=$?
    echo "== $V combine=$C rc=$rc"; grep -v amdgpu.ids gpurun_out/mt.log
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
