# rocprofv3 passes for one workload: kernel trace + stats, then separate PMC passes (HBM bytes, SQ counters), then the
# summary (gpurun_out/prof_<tag>_<workload>/summary.{json,md}; copy to profiles/<tag>_<workload>.* and pmc_<workload>.json).
# usage: bash tools/gpu_prof.sh <workload> <records> <tag>
set +e
W=${1:-tls16k}; N=${2:-262144}; TAG=${3:-r1}
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/prof_${TAG}_${W}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --workload $W --records $N --steps 5 --warmup 1 --extra= --no-cpu-baseline --verify 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- python3 $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o pmc_fetch -- python3 $ARGS > $OUT/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o pmc_write -- python3 $ARGS > $OUT/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT -o pmc_sq -- python3 $ARGS > $OUT/pmc_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL --output-format csv -d $OUT -o pmc_sq2 -- python3 $ARGS > $OUT/pmc_sq2.log 2>&1
rc=$?; echo "pmc sq2 rc=$rc"
python3 $R/tools/prof_summary.py $OUT $OUT/summary $N
exit 0
