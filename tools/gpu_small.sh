# small-batch grid/unit rule and the HP kernel: GPU suite, HP cost, small-batch launches base vs new
set +e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python tools/hp_cost.py > gpurun_out/hp_cost2.log 2>&1; rc=$?; grep hp_cost gpurun_out/hp_cost2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/small_batch.py tools/variants/lib_base.so tools/variants/lib_new.so > gpurun_out/small_batch.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/small_batch.log; exit $rc
