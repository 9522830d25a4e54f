# round 2: the config tests, then the default bench line (all extras + cpu_baseline legs)
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_configs.log 2>&1
rc=$?; echo "pytest configs rc=$rc"; tail -15 gpurun_out/pytest_configs.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py > gpurun_out/bench_r2a.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 6000 gpurun_out/bench_r2a.log
exit $rc
