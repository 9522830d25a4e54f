# round 3: parity tests, then interleaved A/B of the spill reduction (lib_old = round 2, lib_new2 = now) on the BASELINE
# shapes, then rocprofv3 kernel trace + PMC passes (seal and open) for tls16k, quic1200 and mixed with the new build
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_ct.py tests/test_gpu_resources.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
for w in "tls16k 262144" "quic1200 2097152" "mixed 4194304"; do
  set -- $w
  timeout -k 10 300 python tools/ab.py tools/variants/lib_old.so tools/variants/lib_new2.so --workload $1 --records $2 --rounds 5 > gpurun_out/ab_spill_$1.log 2>&1
  rc=$?; echo "ab $1 rc=$rc"; tail -2 gpurun_out/ab_spill_$1.log; [ $rc -ne 0 ] && exit $rc
done
for w in "tls16k 262144" "quic1200 2097152" "mixed 1048576"; do
  set -- $w
  bash tools/gpu_prof.sh $1 $2 r3 > gpurun_out/prof_r3_$1.log 2>&1; rc=$?; echo "prof $1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
