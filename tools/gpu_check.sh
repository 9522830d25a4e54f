set +e
cd $GRAFT_REPO_ROOT
# parity, then schedule matrix, then phase profile (each step bounded; stop at the first failure)
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/sched_matrix.sh > gpurun_out/sched.log 2>&1 || { cat gpurun_out/sched.log; exit 1; }
cat gpurun_out/sched.log
cd tools
for w in "mixed 4194304" "mixed1key 1048576"; do set -- $w; timeout -k 10 200 python prof_phases.py prof/lib_prof.so --workload $1 --records $2 2>&1 | grep -v amdgpu.ids || exit 1; done
