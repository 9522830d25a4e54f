# steady-loop scheduling fences: product (all three) vs without the one after the AES rounds / after the GHASH fold
set +e
V=tools/variants
for w in tls16k_1048576 quic1200_4194304 mixed_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 280 python tools/ab.py $V/sb_111.so $V/sb_011.so $V/sb_110.so --workload $wl --records $n --rounds 3 --reps 2 > gpurun_out/fences_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/fences_$wl.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
done
exit 0
