# early GHASH tables (one-key launches): GPU suite, small-batch launches and per-record latency, noearly vs new
set +e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python tools/small_batch.py tools/variants/lib_base.so tools/variants/lib_new.so > gpurun_out/small_batch.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/small_batch.log; [ $rc -ne 0 ] && exit $rc
LAT_BASE=tools/variants/noearly bash tools/gpu_lat_ab.sh
