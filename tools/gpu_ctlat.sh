#!/bin/bash
# per-record latency: default off / constant-time (old last step) / constant-time (tree), same box
set +e
cd $GRAFT_REPO_ROOT
V=tools/variants
for run in "0 $V/lib_old.so" "1 $V/lib_old.so" "1 $V/lib_both.so" "0 $V/lib_both.so"; do set -- $run
  echo "== PTLS_MI355X_CONSTANT_TIME=$1 $2"
  PTLS_MI355X_CONSTANT_TIME=$1 timeout -k 10 120 python tools/latency.py $2 > gpurun_out/ctlat.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ctlat.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
