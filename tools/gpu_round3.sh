# round-3 check: GPU tests, then the default bench line (all BASELINE configs incl. shard1200)
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -30; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { tail -80 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 6000 gpurun_out/bench_default.log
[ $rc -ne 0 ] && tail -30 gpurun_out/bench_default.err
exit $rc
