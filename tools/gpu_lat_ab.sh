# per-record latency A/B (tools/variants/lib_base.so vs the in-tree build), then the multi-thread per-record rates
set +e
cd $GRAFT_REPO_ROOT
NEW=picotls_amd/_lib/libptls_mi355x.so; BASE=tools/variants/lib_base.so
for i in 1 2; do
  for L in $BASE $NEW; do
    timeout -k 10 120 python tools/latency.py $L > gpurun_out/lat_$i_$(basename $L).log 2>&1; rc=$?
    echo "== $L ($i) rc=$rc"; grep -v amdgpu.ids gpurun_out/lat_$i_$(basename $L).log
    [ $rc -ne 0 ] && exit $rc
  done
done
for L in $BASE $NEW; do
  timeout -k 10 200 python tools/mt_records.py $L > gpurun_out/mt_$(basename $L).log 2>&1; rc=$?
  echo "== mt $L rc=$rc"; grep -v amdgpu.ids gpurun_out/mt_$(basename $L).log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
