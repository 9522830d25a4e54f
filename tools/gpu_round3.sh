# round-3 check: every GPU test, the default bench line (all BASELINE configs incl. shard1200), HP batch cost, the small
# batches with long records
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -30; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { tail -80 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_default.log
[ $rc -ne 0 ] && { tail -30 gpurun_out/bench_default.err; exit $rc; }
timeout -k 10 300 python tools/hp_cost.py --rounds 7 > gpurun_out/hp_cost.txt 2>&1; rc=$?; grep hp_cost gpurun_out/hp_cost.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/small_batch.py --rounds 3 > gpurun_out/small_batch.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/small_batch.txt | head -8
exit $rc
