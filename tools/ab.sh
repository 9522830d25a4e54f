set +e
cd $GRAFT_REPO_ROOT
# usage: tools/ab.sh <workload> <records> [extra ab.py args]
w=${1:-tls16k}; n=${2:-262144}; shift 2
timeout -k 10 400 python tools/ab.py tools/variants/*.so --workload $w --records $n "$@" > gpurun_out/ab_$w.log 2>&1
rc=$?; cat gpurun_out/ab_$w.log | grep -v amdgpu.ids; exit $rc
