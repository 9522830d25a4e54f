# deferred one-key setup: GPU suite, then the lifecycle and latency measurements
set +e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python tools/lifecycle.py > gpurun_out/lifecycle_r2b.log 2>&1; rc=$?; grep "^{" gpurun_out/lifecycle_r2b.log | cut -c1-900; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/latency.py > gpurun_out/latency_r2b.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/latency_r2b.log; exit $rc
