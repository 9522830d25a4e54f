# per-record latency A/B: LAT_BASE (default tools/variants/noflag) vs the in-tree build, interleaved, then the
# multi-thread rates of both at 1200 B
set +e
cd $GRAFT_REPO_ROOT
NEW=${LAT_NEW:-picotls_amd/_lib}; BASE=${LAT_BASE:-tools/variants/noflag}
for i in 1 2; do
  for L in $BASE $NEW; do
    timeout -k 10 120 python tools/latency.py $L/libptls_mi355x.so > gpurun_out/lat.log 2>&1; rc=$?
    echo "== $L ($i) rc=$rc"; grep -v amdgpu.ids gpurun_out/lat.log
    [ $rc -ne 0 ] && exit $rc
  done
done
for L in $BASE $NEW; do
  LD_LIBRARY_PATH=$L timeout -k 10 120 tools/_bin/mt_records 0.5 1200 > gpurun_out/mt.log 2>&1; rc=$?
  echo "== mt $L rc=$rc"; grep -v amdgpu.ids gpurun_out/mt.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
