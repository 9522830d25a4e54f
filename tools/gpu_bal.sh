# byte-balanced workgroup ranges for many-key batches: GPU suite, then interleaved A/B (BALANCE=0 vs 1)
set +e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh || exit 1
V="tools/variants/lib_nobal.so tools/variants/lib_bal.so"
for w in "mixedconn 4194304" "mixed 4194304" "mixedrand 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py $V --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$1.log | tail -3; [ $rc -ne 0 ] && exit $rc
done
exit 0
