# rocprofv3 kernel stats + VALU/LDS counters of the T-table vs bitsliced AES-CTR microbenchmark
set +e
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/prof_aesctr
mkdir -p $OUT
timeout -k 10 120 python3 $R/tools/mb/aes_ctr.py > $OUT/run128.log 2>&1 && cat $OUT/run128.log || exit 1
timeout -k 10 120 python3 $R/tools/mb/aes_ctr.py --key-size 32 > $OUT/run256.log 2>&1 && cat $OUT/run256.log || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- python3 $R/tools/mb/aes_ctr.py > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT -o pmc -- python3 $R/tools/mb/aes_ctr.py > $OUT/pmc.log 2>&1
echo "pmc rc=$?"
cat $OUT/trace_kernel_stats.csv | cut -c1-200
