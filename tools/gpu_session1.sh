set +e
cd $GRAFT_REPO_ROOT
nproc; grep -m1 "model name" /proc/cpuinfo; grep -c processor /proc/cpuinfo; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --records 262144 --steps 5 --warmup 1 --extra quic1200 --cpu-seconds 2 > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench_small.log
exit $rc
