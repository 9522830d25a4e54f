# GPU parity tests only (bounded), optionally a test-file filter: bash tools/gpu_tests.sh [pytest args]
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -60; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && tail -60 gpurun_out/pytest_gpu.log
exit $rc
