#!/bin/bash
# round-6 GPU steps: bash tools/gpu_r6.sh <step> ...   (each step bounded; results under gpurun_out/)
set +e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    final) bash tools/gpu_final.sh r6a || exit $? ;;
    t_*)  # t_<pytest -k expression>: the gpu tests whose names match
      k=${step#t_}
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$k" > gpurun_out/t_$k.log 2>&1
      rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t_$k.log | tail -25; [ $rc -ne 0 ] && exit $rc ;;
    ab_*)  # ab_<workload>_<records>: interleaved A/B of tools/abv/*.so
      w=$(echo $step | cut -d_ -f2); n=$(echo $step | cut -d_ -f3)
      timeout -k 10 500 python tools/ab.py tools/abv/*.so --workload $w --records $n --rounds 5 > gpurun_out/ab_$w.log 2>&1 || { cat gpurun_out/ab_$w.log | tail -20; exit 1; }
      grep -v amdgpu.ids gpurun_out/ab_$w.log | tail -12 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
