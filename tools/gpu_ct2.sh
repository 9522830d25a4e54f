# the constant-time evidence with the product build: LDS counters of the seal/open kernels, default and CT mode, for two
# keys x two payloads on tls16k, quic1200 and mixed (one rocprofv3 pass per process), then the CT cost (tools/ab.py, ":ct" variants)
set +e
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for wn in "tls16k 65536" "quic1200 262144" "mixed 262144"; do set -- $wn
for mode in default ct; do flag=""; [ $mode = ct ] && flag="--ct"
for k in 1 2; do for pl in zero random; do
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/ct3/$1_${mode}_k${k}_$pl -o p -- python3 $R/tools/ct_probe.py $flag --workload $1 --records $2 --key-seed $k --payload $pl > $R/gpurun_out/ct3_$1_${mode}_k${k}_$pl.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$1 $mode $k $pl rc=$rc"; tail -5 $R/gpurun_out/ct3_$1_${mode}_k${k}_$pl.log; exit $rc; }
done; done; done; echo "$1 done"; done
cd $R
L=picotls_amd/_lib/libptls_mi355x.so
for w in tls16k_1048576 quic1200_4194304 mixed_4194304; do set -- ${w/_/ }
  timeout -k 10 300 python tools/ab.py $L $L:ct --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/abct_$1.log 2>&1
  rc=$?; echo "== $1"; grep -v amdgpu.ids gpurun_out/abct_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
