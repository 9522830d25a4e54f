# scheduler-flag sweep of the whole engine build (tools/ab.py, interleaved, identical output checked)
set +e
V=tools/variants
L="$V/v0_base.so $V/v1_trackers.so $V/v2_nohighrp.so $V/v3_maxilp.so $V/v4_memclause.so $V/v5_minreg.so"
for w in tls16k_262144 quic1200_1048576 mixed_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 280 python tools/ab.py $L --workload $wl --records $n --rounds 3 --reps 2 > gpurun_out/flags_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/flags_$wl.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
done
exit 0
