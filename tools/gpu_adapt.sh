# per-run unit length chosen by the scan (run_unit_log2) vs the host rule: big-batch A/B, small batches, per-record
# latency, GPU suite
set +e
A=tools/variants/lib_base.so; B=tools/variants/lib_adapt.so
for w in tls16k_262144 quic1200_1048576 mixed_4194304 mixedrand_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 250 python tools/ab.py $A $B --workload $wl --records $n --rounds 4 --reps 2 > gpurun_out/adapt_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/adapt_$wl.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/small_batch.py $A $B --rounds 3 > gpurun_out/adapt_small.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/adapt_small.log | cut -c1-120; [ $rc -ne 0 ] && exit $rc
for L in $A $B; do timeout -k 10 200 python tools/latency.py $L > gpurun_out/adapt_lat_$(basename $L .so).log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/adapt_lat_$(basename $L .so).log; [ $rc -ne 0 ] && exit $rc; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; exit $rc
