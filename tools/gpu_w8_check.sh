bash tools/gpu_recipes.sh lasterr 15 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_w8.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/w8_product.log 2>&1; rc=$?
echo "product build test_gpu_w8 rc=$rc"; tail -3 gpurun_out/w8_product.log; [ $rc -ne 0 ] && { tail -40 gpurun_out/w8_product.log; exit $rc; }
PTLS_MI355X_LIB=$PWD/tools/variants/lib_w8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_w8.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_ct.py -m gpu -x -v --timeout 120 --timeout-method thread -k "not vtable" > gpurun_out/w8_variant.log 2>&1; rc=$?
echo "W8 variant suite rc=$rc"; grep -cE "PASSED" gpurun_out/w8_variant.log; tail -3 gpurun_out/w8_variant.log; [ $rc -ne 0 ] && tail -60 gpurun_out/w8_variant.log
exit $rc
