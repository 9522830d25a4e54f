# AES table copy with 8 loads in flight per thread (vs 4): GPU suite, small-batch launches and per-record latency A/B,
# bulk A/B
set +e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh -k "first_run or per_record or fuzz" || exit 1
timeout -k 10 300 python tools/small_batch.py tools/variants/lib_base.so tools/variants/lib_new.so > gpurun_out/small_batch.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/small_batch.log; [ $rc -ne 0 ] && exit $rc
for w in "tls16k 1048576" "quic1200 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py tools/variants/lib_base.so tools/variants/lib_new.so --workload $1 --records $2 --rounds 3 --reps 2 > gpurun_out/ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$1.log | tail -2; [ $rc -ne 0 ] && exit $rc
done
LAT_BASE=tools/variants/b4 LAT_NEW=tools/variants/b8 bash tools/gpu_lat_ab.sh
