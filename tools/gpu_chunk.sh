# unit size A/B: 2 KiB (product) vs 4 KiB units on the mixed-length workloads (identical output checked by tools/ab.py)
set +e
A=tools/variants/lib_c128.so; B=tools/variants/lib_c256.so
for w in mixed_4194304 mixed1key_1048576 mixedrand_4194304 quic1200_1048576; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 250 python tools/ab.py $A $B --workload $wl --records $n --rounds 4 --reps 2 > gpurun_out/chunk_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/chunk_$wl.log | cut -c1-175; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/small_batch.py $A $B --rounds 3 > gpurun_out/chunk_small.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/chunk_small.log; exit $rc
