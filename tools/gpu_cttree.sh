#!/bin/bash
# constant-time tree A/B: parity of the CT paths, then default vs CT (old four-multiply last step, lane tree, lane tree +
# combine tree) in one process per workload
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ct.py tests/test_gpu_resources.py > gpurun_out/cttree_tests.log 2>&1
rc=$?; tail -3 gpurun_out/cttree_tests.log; [ $rc -ne 0 ] && exit $rc
V=tools/variants
for w in tls16k_1048576 quic1200_4194304 mixed_4194304; do set -- ${w/_/ }
  timeout -k 10 300 python tools/ab.py $V/lib_old.so $V/lib_old.so:ct $V/lib_tree.so:ct $V/lib_both.so:ct --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/cttree_$1.log 2>&1
  rc=$?; echo "== $1"; grep -v amdgpu.ids gpurun_out/cttree_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
