# round 2: the whole GPU suite, then the lifecycle measurement
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15
[ $rc -ne 0 ] && { tail -80 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python tools/lifecycle.py > gpurun_out/lifecycle.log 2>&1
rc=$?; echo "lifecycle rc=$rc"; tail -5 gpurun_out/lifecycle.log
exit $rc
