set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_full.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify 0 > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log
find $GRAFT_REPO_ROOT/gpurun_out/prof_r1 -name "*stats*" | head
exit $rc
