# round 3: long records in small one-key batches over many workgroups (spread_pieces) -- parity, small-batch timing
# against the build before, bulk A/B
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lifecycle.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python tools/small_batch.py tools/variants/lib_prespread.so tools/variants/lib_spread.so --rounds 4 > gpurun_out/small_spread.txt 2>&1; rc=$?; echo "small rc=$rc"; grep -v amdgpu gpurun_out/small_spread.txt | tail -40; [ $rc -ne 0 ] && exit $rc
for w in "quic1200 4194304" "tls16k 262144" "mixed 4194304"; do
  set -- $w
  timeout -k 10 300 python tools/ab.py tools/variants/lib_prespread.so tools/variants/lib_spread.so --workload $1 --records $2 --rounds 4 > gpurun_out/ab_spread_$1.log 2>&1
  rc=$?; echo "ab $1 rc=$rc"; tail -2 gpurun_out/ab_spread_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
