# round 3: constant-time evidence of the per-record path (picotls objects, CT by default) and its latency phases
set +e
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for ln in 1200 16384 1048576; do
for mode in ct nonct; do env=""; [ $mode = nonct ] && export PTLS_MI355X_CONSTANT_TIME=0 || unset PTLS_MI355X_CONSTANT_TIME
for k in 1 2; do for pl in zero random; do
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/ctpr/${ln}_${mode}_k${k}_$pl -o p -- python3 $R/tools/ct_probe_perrec.py --len $ln --key-seed $k --payload $pl --calls 4 > $R/gpurun_out/ctpr_${ln}_${mode}_k${k}_$pl.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$ln $mode $k $pl rc=$rc"; tail -5 $R/gpurun_out/ctpr_${ln}_${mode}_k${k}_$pl.log; exit $rc; }
done; done; done; echo "$ln done"; done
unset PTLS_MI355X_CONSTANT_TIME
cd $R
python3 tools/ct_summary.py gpurun_out/ctpr > gpurun_out/ct_perrec.txt; cat gpurun_out/ct_perrec.txt | head -80
for ln in 1200 16384; do
  timeout -k 10 120 python tools/lat_one.py $ln tools/variants/lib_prof.so > gpurun_out/phase_ct_$ln.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/phase_ct_$ln.txt; [ $rc -ne 0 ] && exit $rc
  PTLS_MI355X_CONSTANT_TIME=0 timeout -k 10 120 python tools/lat_one.py $ln tools/variants/lib_prof.so > gpurun_out/phase_nonct_$ln.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/phase_nonct_$ln.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
