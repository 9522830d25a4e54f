# steady range one step longer (clamped last prefetch) vs the product build: A/B on the bench workloads, then the GPU
# parity tests of the variant's code paths run against the variant (PTLS_MI355X_LIB is not a thing: the A/B checks
# identical output with tools/ab.py)
set +e
A=tools/variants/lib_base.so; B=tools/variants/lib_sext.so
for w in tls16k_1048576 quic1200_4194304 mixed_4194304 mixedrand_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 280 python tools/ab.py $A $B $A:ct $B:ct --workload $wl --records $n --rounds 3 --reps 2 > gpurun_out/sext_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/sext_$wl.log | cut -c1-170; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/small_batch.py $A $B --rounds 3 > gpurun_out/sext_small.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/sext_small.log | cut -c1-120; exit $rc
