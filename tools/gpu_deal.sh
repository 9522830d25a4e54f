# chunk dealing (CHUNKS_PER_WG 0 = contiguous ranges, 4, 8, 16): GPU parity suite, then interleaved A/B at bench sizes
set +e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh || exit 1
V="tools/variants/lib_k0.so tools/variants/lib_k4.so tools/variants/lib_k8.so tools/variants/lib_k16.so"
for w in "mixedsorted 4194304" "tls16k 1048576" "quic1200 4194304" "mixed 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py $V --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$1.log | tail -8; [ $rc -ne 0 ] && exit $rc
done
exit 0
