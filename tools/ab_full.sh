# full-size interleaved A/B of tools/variants/*.so on the two headline configs
set +e
cd $GRAFT_REPO_ROOT
for w in ${AB_WORKLOADS:-tls16k_1048576 quic1200_4194304}; do set -- ${w/_/ }
timeout -k 10 300 python tools/ab.py tools/variants/*.so --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/abf_$1.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/abf_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
