# full measurement session: default bench (+e2e), the many-key config and the 32M x 1200 B config on one GPU
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --e2e > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench default rc=$rc"; grep "^{" gpurun_out/bench_default.log | tail -1 | cut -c1-3000
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_default.log; exit $rc; }
timeout -k 10 600 python bench.py --workload mixed --extra= --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_mixed.log 2>&1
rc=$?; echo "bench mixed rc=$rc"; grep "^{" gpurun_out/bench_mixed.log | tail -1 | cut -c1-1500
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_mixed.log; exit $rc; }
timeout -k 10 600 python bench.py --workload mixedrand --extra= --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_mixedrand.log 2>&1
rc=$?; echo "bench mixedrand rc=$rc"; grep "^{" gpurun_out/bench_mixedrand.log | tail -1 | cut -c1-1500
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_mixedrand.log; exit $rc; }
timeout -k 10 600 python bench.py --workload shard1200 --extra= --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_shard.log 2>&1
rc=$?; echo "bench shard1200 rc=$rc"; grep "^{" gpurun_out/bench_shard.log | tail -1 | cut -c1-1500
exit $rc
