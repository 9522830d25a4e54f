# round 3: header protection fused into the seal launch -- parity, batch cost, plain-seal A/B against the build before
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lifecycle.py tests/test_gpu_resources.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
for r in 1 2; do
timeout -k 10 300 python tools/hp_cost.py --rounds 7 > gpurun_out/hp_cost_$r.txt 2>&1; rc=$?; echo "hp_cost rc=$rc"; grep hp_cost gpurun_out/hp_cost_$r.txt; [ $rc -ne 0 ] && exit $rc
done
for w in "quic1200 4194304" "tls16k 262144"; do
  set -- $w
  timeout -k 10 300 python tools/ab.py tools/variants/lib_prehp.so tools/variants/lib_hpfused.so --workload $1 --records $2 --rounds 5 > gpurun_out/ab_hp_$1.log 2>&1
  rc=$?; echo "ab $1 rc=$rc"; tail -2 gpurun_out/ab_hp_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
