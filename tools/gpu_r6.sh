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
    rcal)  # FETCH_SIZE / WRITE_SIZE per byte for the quad load shapes (tools/mb/wcal.hip), 1M packed 1216-byte records
      ( R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out/rcal
        for spec in "ld_m0 FETCH_SIZE 0 1" "ld_m1 FETCH_SIZE 1 1" "ld_m2 FETCH_SIZE 2 1" "ld_m4 FETCH_SIZE 4 1" "ld_m5 FETCH_SIZE 5 1" \
                    "st_m0 WRITE_SIZE 0 0" "st_m4 WRITE_SIZE 4 0" "st_m5 WRITE_SIZE 5 0"; do
          set -- $spec
          timeout -k 10 120 rocprofv3 --pmc $2 --output-format csv -d $R/gpurun_out/rcal/$1 -o p -- $R/tools/mb/wcal.bin $3 $4 1048576 1216 200 3 > $R/gpurun_out/rcal/$1.log 2>&1 || exit 1
        done )
      rc=$?; python3 tools/wcal_summary.py gpurun_out/rcal; [ $rc -ne 0 ] && exit $rc ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
