# recomputed lane index (fewer scratch spills): A/B on every bench workload, default and constant-time, then the GPU suite
set +e
A=tools/variants/lib_base.so; B=tools/variants/lib_lane.so
for w in tls16k_1048576 quic1200_4194304 mixed_4194304 mixedrand_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 280 python tools/ab.py $A $B $A:ct $B:ct --workload $wl --records $n --rounds 3 --reps 2 > gpurun_out/lane_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/lane_$wl.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/small_batch.py $A $B --rounds 3 > gpurun_out/lane_small.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/lane_small.log | cut -c1-120; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; exit $rc
