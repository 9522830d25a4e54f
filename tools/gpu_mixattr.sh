# where the mixed-length many-key line loses against uniform records: the product build on AES-256
# workloads of ~4 GiB payload: uniform 16 KiB, uniform 8 KiB (the mixed mean), mixed lengths under one key, and the
# configs[3] batch itself (64K keys, full size so that every key has its 64 records)
set +e
L=picotls_amd/_lib/libptls_mi355x.so
for w in tls16k256_262144 u8k256_524288 mixed1key_524288 mixed_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 200 python tools/ab.py $L --workload $wl --records $n --rounds 3 --reps 2 > gpurun_out/mixattr_$wl.log 2>&1
  rc=$?; echo "== $wl"; grep -v amdgpu.ids gpurun_out/mixattr_$wl.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
