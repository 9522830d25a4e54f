# attribution passes: WRITE_SIZE of the seal for two output layouts (tools/write_align.py), then the constant-time probe
# (tools/ct_probe.py) under two keys x {zero, random} payloads with the LDS counters; one rocprofv3 pass per process
set +e
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for lay in packed aligned; do
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/attrib/$lay -o p -- python3 $R/tools/write_align.py --layout $lay > $R/gpurun_out/attrib_$lay.log 2>&1
  rc=$?; echo "layout $lay rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/attrib_$lay.log; exit $rc; }
done
for k in 1 2; do for pl in zero random; do
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/ct/k${k}_$pl -o p -- python3 $R/tools/ct_probe.py --key-seed $k --payload $pl > $R/gpurun_out/ct_k${k}_$pl.log 2>&1
  rc=$?; echo "ct key $k $pl rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/ct_k${k}_$pl.log; exit $rc; }
done; done
exit 0
