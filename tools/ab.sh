set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/ab.py tools/variants/*.so --workload ${1:-tls16k} --records ${2:-262144} > gpurun_out/ab.log 2>&1
rc=$?; cat gpurun_out/ab.log | grep -v amdgpu.ids; exit $rc
