# round 2 checkpoint: GPU suite, default bench line, rocprofv3 summaries of the three bench workloads (tag r2)
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 500 python bench.py > gpurun_out/bench_r2f.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/bench_r2f.log | cut -c1-600; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r2f.log; exit $rc; }
for w in "tls16k 1048576" "quic1200 4194304" "mixed 4194304"; do set -- $w
  bash tools/gpu_prof.sh $1 $2 r2 || exit 1
done
exit 0
