# phase breakdown of the chunked kernel (ENGINE_PROFILE build): a lone record, a 1000-record batch, the bench batches
set +e
cd tools
for w in "tls16k 1" "tls16k 1000" "quic1200 1000" "tls16k 262144" "mixed 4194304" "mixed1key 1048576"; do set -- $w
  timeout -k 10 200 python prof_phases.py variants/lib_prof.so --workload $1 --records $2 --reps 5 2>&1 | grep -v amdgpu.ids || exit 1
done
exit 0
