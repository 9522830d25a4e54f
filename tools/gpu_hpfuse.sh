# fused per-record header protection: GPU suite, bulk A/B (previous build vs this one), per-record latency A/B
set +e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh || exit 1
V="tools/variants/lib_prev.so tools/variants/lib_new.so"
for w in "tls16k 1048576" "quic1200 4194304" "mixed 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py $V --workload $1 --records $2 --rounds 3 --reps 2 > gpurun_out/ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$1.log | tail -2; [ $rc -ne 0 ] && exit $rc
done
LAT_BASE=tools/variants/nofuse bash tools/gpu_lat_ab.sh
