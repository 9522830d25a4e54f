# HBM bytes (FETCH_SIZE / WRITE_SIZE, separate rocprofv3 passes) of each tools/variants/*.so on one workload:
# bash tools/pmc_variants.sh <workload> <records>
set +e
W=${1:-tls16k}; N=${2:-262144}
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for lib in $R/tools/variants/*.so; do v=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmcv/$v/$c -o p -- python3 $R/tools/ab.py $lib --workload $W --records $N --rounds 1 --reps 1 > $R/gpurun_out/pmcv_${v}_$c.log 2>&1
    rc=$?; echo "$v $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/pmcv_${v}_$c.log; exit $rc; }
  done
done
exit 0
