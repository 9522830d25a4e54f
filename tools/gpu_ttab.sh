# AES T-table copied from a compile-time image vs derived per launch: small batches, a lone record, bulk, phases, GPU suite
set +e
A=tools/variants/lib_derive.so; B=tools/variants/lib_copy.so
timeout -k 10 300 python tools/small_batch.py $A $B --rounds 3 > gpurun_out/ttab_small.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ttab_small.log | cut -c1-130; [ $rc -ne 0 ] && exit $rc
for w in tls16k_1048576 quic1200_4194304 mixed_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 280 python tools/ab.py $A $B --workload $wl --records $n --rounds 3 --reps 2 > gpurun_out/ttab_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/ttab_$wl.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 python tools/latency.py > gpurun_out/ttab_lat.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ttab_lat.log; [ $rc -ne 0 ] && exit $rc
cd tools
for w in "tls16k 1" "tls16k 1000" "quic1200 1000" "tls16k 262144" "mixed 4194304"; do set -- $w
  timeout -k 10 200 python prof_phases.py variants/lib_prof.so --workload $1 --records $2 --reps 5 2>&1 | grep -v amdgpu.ids || exit 1
done
cd ..
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; exit $rc
