# many-key mixed seal traffic attribution (tools/mixed_align.py): per layout a timing run, then one rocprofv3 --pmc
# pass each for WRITE_SIZE and FETCH_SIZE (one TCC counter group per pass)
set +e
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for lay in packed slot128 lines; do
  timeout -k 10 150 python3 $R/tools/mixed_align.py --layout $lay --reps 4 > $R/gpurun_out/mixalign_$lay.log 2>&1
  rc=$?; echo "== $lay rc=$rc"; grep mixed_align $R/gpurun_out/mixalign_$lay.log; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/mixalign_$lay.log; exit $rc; }
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -k 10 150 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/mixalign/${lay}_$c -o p -- python3 $R/tools/mixed_align.py --layout $lay --reps 2 > $R/gpurun_out/mixalign_${lay}_$c.log 2>&1
    rc=$?; echo "$lay $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/mixalign_${lay}_$c.log; exit $rc; }
  done
done
exit 0
