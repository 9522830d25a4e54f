# constant-time probe of each tools/variants/*.so: LDS counters of the seal/open kernels under two keys x two payloads
# (one rocprofv3 pass per process), then the interleaved A/B of the variants
set +e
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
W=${CT_WORKLOAD:-tls16k}; N=${CT_RECORDS:-65536}
for lib in $R/tools/variants/*.so; do v=$(basename $lib .so)
for k in 1 2; do for pl in zero random; do
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/ct2/$v/${W}_k${k}_$pl -o p -- python3 $R/tools/ct_probe.py --lib $lib --workload $W --records $N --key-seed $k --payload $pl > $R/gpurun_out/ct2_${v}_k${k}_$pl.log 2>&1
  rc=$?; echo "$v key $k $pl rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/ct2_${v}_k${k}_$pl.log; exit $rc; }
done; done; done
cd $R && bash tools/ab_three.sh
