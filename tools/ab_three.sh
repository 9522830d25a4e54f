# interleaved A/B of tools/variants/*.so on tls16k, quic1200 and the 64K-key mixed config at full size
set +e
cd $GRAFT_REPO_ROOT
for w in ${AB_WORKLOADS:-tls16k_1048576 quic1200_4194304 mixed_4194304}; do set -- ${w/_/ }
timeout -k 10 300 python tools/ab.py tools/variants/*.so --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/ab_$1.log 2>&1
rc=$?; echo "== $1"; grep -v amdgpu.ids gpurun_out/ab_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
