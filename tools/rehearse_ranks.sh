# 2- and 4-rank rehearsal of bench.py's distributed path on one GPU (all ranks on cuda:0, gloo reductions):
# checks the launch, sharding, barrier/max timing and the rank-0 JSON line, not scaling.
set +e
cd $GRAFT_REPO_ROOT
export PTLS_BENCH_ONE_DEVICE=1
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) \
      bench.py --gpus $n --steps 3 --warmup 1 --records 32768 --extra quic1200 > gpurun_out/rehearse_$n.log 2>&1
  rc=$?; echo "ranks=$n rc=$rc"; grep '^{' gpurun_out/rehearse_$n.log | cut -c1-400
  [ $rc -ne 0 ] && { tail -20 gpurun_out/rehearse_$n.log; exit $rc; }
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) \
      bench.py --gpus $n --steps 3 --warmup 1 --workload shard1200 --records 262144 --extra= > gpurun_out/rehearse_shard_$n.log 2>&1
  rc=$?; echo "ranks=$n shard1200 rc=$rc"; grep '^{' gpurun_out/rehearse_shard_$n.log | cut -c1-400
  [ $rc -ne 0 ] && { tail -20 gpurun_out/rehearse_shard_$n.log; exit $rc; }
done
exit 0
