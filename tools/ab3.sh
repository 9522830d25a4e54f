set +e
cd $GRAFT_REPO_ROOT
for w in "tls16k 262144" "quic1200 2097152" "mixed 1048576"; do set -- $w
timeout -k 10 300 python tools/ab.py tools/variants/lib_base.so tools/variants/lib_cache1.so --workload $1 --records $2 > gpurun_out/ab_$1.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
