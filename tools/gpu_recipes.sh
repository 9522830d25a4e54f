#!/bin/bash
# The one-off GPU measurement recipes of rounds 2-3 (interleaved A/Bs of engine variants, counter passes, latency
# sweeps), kept in one file so that the profiles/ files they produced can name their source:
#   bash tools/gpu_recipes.sh <name>    (run on the GPU box through gpurun, from the repository root)
# Variant libraries (tools/variants/*.so) are built beforehand with tools/mkvariant.sh (and ./tools/variants taken out of
# .gpurunignore for the calls that use them: it is listed there so that ordinary GPU calls do not carry them); the recurring drivers stay
# separate: tools/gpu_tests.sh (GPU parity suite), tools/gpu_prof.sh (rocprofv3 passes), tools/gpu_mt.sh and
# tools/gpu_lat_ab.sh (per-record rates and latency), tools/ab.sh / tools/ab.py (A/B of variants).
set +e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
recipe=$1; shift
case "$recipe" in
prof4)
  # round 4, the shipped build (W8 on, constant-time default) at the full BASELINE sizes: kernel trace + stats and the
  # separate PMC passes of tools/gpu_prof.sh for each batch config
  (
for wn in "tls16k 1048576" "quic1200 4194304" "mixed 4194304"; do set -- $wn
  bash tools/gpu_prof.sh $1 $2 r4 || exit $?
done
exit 0
  )
  ;;
ct5)
  # round 4: every keyset constant-time by default; LDS counters of the batch kernels at the full BASELINE sizes for
  # two keys x two payloads (one rocprofv3 pass per process, 2 dispatches each of seal and open)
  (
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for wn in "tls16k 1048576" "quic1200 4194304" "mixed 4194304"; do set -- $wn
for k in 1 2; do for pl in zero random; do
  timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/ct5/$1_k${k}_$pl -o p -- python3 $R/tools/ct_probe.py --workload $1 --records $2 --key-seed $k --payload $pl --reps 2 > $R/gpurun_out/ct5_$1_k${k}_$pl.log 2>&1
  rc=$?; echo "$1 $k $pl rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/ct5_$1_k${k}_$pl.log; exit $rc; }
done; done; done
cd $R
python3 tools/ct_summary.py gpurun_out/ct5 > gpurun_out/ct5_batch.txt; cat gpurun_out/ct5_batch.txt
exit 0
  )
  ;;
coh)
  # round 4: per-record latency with coarse-grained (HIP default) vs coherent staging buffers, alternating processes,
  # then the spread and lifecycle tests with the batch-sized spread scratch
  (
for i in 1 2 3; do for c in 0 1; do
  PTLS_MI355X_STAGE_COHERENT=$c timeout -k 10 120 python tools/latency.py > gpurun_out/coh_${c}_$i.log 2>&1; rc=$?
  echo "== coherent=$c run $i rc=$rc"; grep -v amdgpu.ids gpurun_out/coh_${c}_$i.log | head -12; [ $rc -ne 0 ] && exit $rc
done; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_lifecycle.py tests/test_gpu_w8.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/coh_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/coh_tests.log; exit $rc
  )
  ;;
trace2)
  # kernel trace of tools/ab.py with one library each (args: lib1 lib2 workload records)
  (
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for L in $1 $2; do n=$(basename $L .so)
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace2_$n -o t -- python3 $R/tools/ab.py $R/$L --workload $3 --records $4 --rounds 3 --reps 2 > $R/gpurun_out/trace2_$n.log 2>&1
  rc=$?; echo "== $n rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/trace2_$n.log; exit $rc; }
  f=$(ls $R/gpurun_out/trace2_$n/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && cut -d, -f1-6 $f | head -8
done
exit 0
  )
  ;;
w8all)
  # round 4: every run of an unframed batch in the W8 kernel alone (lib_w8all) against the shipped pair (lib_base4)
  # and W8 cut runs in the reordered pair (lib_w8cut_rev): parity of the new variant, bulk A/B, small batches
  (
PTLS_MI355X_LIB=$PWD/tools/variants/${W8ALL_LIB:-lib_w8all.so} timeout -k 10 600 python -u -m pytest tests/test_gpu_w8.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_ct.py tests/test_gpu_lifecycle.py tests/test_gpu_tls12.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not vtable" > gpurun_out/w8all_tests.log 2>&1; rc=$?
echo "w8all suite rc=$rc"; tail -3 gpurun_out/w8all_tests.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/w8all_tests.log | head -80; exit $rc; }
V=${W8ALL_AB:-"tools/variants/lib_base4.so tools/variants/lib_w8cut_rev.so tools/variants/lib_w8all.so"}
for w in "mixed 4194304" "mixedrand 4194304" "mixedconn 4194304" "mixed1key 2097152" "tls16k 1048576" "quic1200 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py $V --workload $1 --records $2 --rounds 6 --reps 2 > gpurun_out/w8all_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/w8all_$1.log | tail -3 | cut -c1-150; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/small_batch.py tools/variants/lib_base4.so tools/variants/${W8ALL_LIB:-lib_w8all.so} --rounds 3 > gpurun_out/w8all_small.log 2>&1; rc=$?
echo "== small batches rc=$rc"; grep -v amdgpu.ids gpurun_out/w8all_small.log | tail -30
exit $rc
  )
  ;;
w8ab)
  # round 4: the 8-bit Horner table (W8_HORNER=1, tools/variants/lib_w8.so) against the same source without it
  # (lib_now8.so), interleaved in one process per workload (tools/ab.py: identical sealed output checked)
  (
V="tools/variants/lib_now8.so tools/variants/lib_w8.so"
for w in "tls16k 1048576" "quic1200 4194304" "mixed 4194304" "mixedrand 4194304" "tls16k256 524288" "mixed1key 2097152"; do set -- $w
  timeout -k 10 300 python tools/ab.py $V --workload $1 --records $2 --rounds 6 --reps 2 > gpurun_out/w8ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/w8ab_$1.log | tail -3; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
lasterr)
  # HIP last-error semantics (tools/mb/lasterr.hip), then the full C vtable suite N times in fresh processes with the
  # round-3 engine (its TLS 1.2 failure of GPUTEST_r03 came in one of three such processes)
  (
timeout -k 10 60 tools/variants/lasterr || exit $?
N=${1:-20}; f=0
for i in $(seq 1 $N); do
  LD_LIBRARY_PATH=$PWD/tools/variants/r3 PTLS_MI355X_COMBINE=4 timeout -k 10 120 tests/c/_bin/test_vtable > gpurun_out/lasterr_r3_$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { f=$((f+1)); echo "== run $i rc=$rc"; grep -E '^(not ok|#)' gpurun_out/lasterr_r3_$i.log | head -20; }
  [ $rc -gt 1 ] && exit $rc
done
echo "r3 full suite: $f of $N runs failed"
exit 0
  )
  ;;
race)
  # round 4: the TLS 1.2 per-record failure of GPUTEST_r03 (test_vtable.c:261-262). Back-to-back 16 KiB per-record
  # calls (test_vtable stress N) with the round-3 engine (tools/variants/r3, built from the round-3 sources), this
  # engine with coarse-grained staging (PTLS_MI355X_STAGE_COHERENT=0) and this engine as shipped; then the full C suite
  (
B=tests/c/_bin/test_vtable; N=${1:-3000}
for v in r3 coarse new; do
  case $v in
  r3) LD_LIBRARY_PATH=$PWD/tools/variants/r3 timeout -k 10 240 $B stress $N > gpurun_out/race_$v.log 2>&1; rc=$? ;;
  coarse) PTLS_MI355X_STAGE_COHERENT=0 timeout -k 10 240 $B stress $N > gpurun_out/race_$v.log 2>&1; rc=$? ;;
  new) timeout -k 10 240 $B stress $N > gpurun_out/race_$v.log 2>&1; rc=$? ;;
  esac
  echo "== $v rc=$rc"; grep '^#' gpurun_out/race_$v.log | tail -14
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
timeout -k 10 300 $B > gpurun_out/race_full.log 2>&1; rc=$?; echo "== full suite rc=$rc"; tail -3 gpurun_out/race_full.log
exit $rc
  )
  ;;
bal)
  # byte-balanced workgroup ranges for many-key batches: GPU suite, then interleaved A/B (BALANCE=0 vs 1)
  (
bash tools/gpu_tests.sh || exit 1
V="tools/variants/lib_nobal.so tools/variants/lib_bal.so"
for w in "mixedconn 4194304" "mixed 4194304" "mixedrand 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py $V --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$1.log | tail -3; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
chunk)
  # unit size A/B: 2 KiB (product) vs 4 KiB units on the mixed-length workloads (identical output checked by tools/ab.py)
  (
A=tools/variants/lib_c128.so; B=tools/variants/lib_c256.so
for w in mixed_4194304 mixed1key_1048576 mixedrand_4194304 quic1200_1048576; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 250 python tools/ab.py $A $B --workload $wl --records $n --rounds 4 --reps 2 > gpurun_out/chunk_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/chunk_$wl.log | cut -c1-175; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/small_batch.py $A $B --rounds 3 > gpurun_out/chunk_small.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/chunk_small.log; exit $rc
  )
  ;;
combtab)
  # unit combine gmul_group (default) vs gmul_tab: interleaved A/B, then LDS bank conflicts of each on the mixed seal
  (
V="tools/variants/lib_group.so tools/variants/lib_tab.so"
for w in "mixed 4194304" "mixedrand 4194304" "quic1200 4194304" "mixedsorted 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py $V --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$1.log | tail -3; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
ct2)
  # the constant-time evidence with the product build: LDS counters of the seal/open kernels, default and CT mode, for two
  # keys x two payloads on tls16k, quic1200 and mixed (one rocprofv3 pass per process), then the CT cost (tools/ab.py, ":ct" variants)
  (
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
  )
  ;;
coop)
  # round 3: window-major power tables (coop_last_powers, gmul_group_w): GPU suite, then the LDS counters of the default
  # mode for two keys x two payloads (batch kernels: tls16k, quic1200, mixed), and of both modes for per-record calls
  (
bash tools/gpu_tests.sh || exit 1
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for wn in "tls16k 65536" "quic1200 262144" "mixed 262144"; do set -- $wn
for k in 1 2; do for pl in zero random; do
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/ct4/$1_default_k${k}_$pl -o p -- python3 $R/tools/ct_probe.py --workload $1 --records $2 --key-seed $k --payload $pl > $R/gpurun_out/ct4_$1_k${k}_$pl.log 2>&1
  rc=$?; echo "$1 $k $pl rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/ct4_$1_k${k}_$pl.log; exit $rc; }
done; done; done
for mode in ct default; do [ $mode = default ] && export PTLS_MI355X_CONSTANT_TIME=0 || unset PTLS_MI355X_CONSTANT_TIME
for ln in 1200 16384 1048576; do
for k in 1 2; do for pl in zero random; do
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/ct4pr/${ln}_${mode}_k${k}_$pl -o p -- python3 $R/tools/ct_probe_perrec.py --len $ln --key-seed $k --payload $pl --calls 4 > $R/gpurun_out/ct4pr_${ln}_${mode}_k${k}_$pl.log 2>&1
  rc=$?; echo "$ln $mode $k $pl rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/ct4pr_${ln}_${mode}_k${k}_$pl.log; exit $rc; }
done; done; done; done
unset PTLS_MI355X_CONSTANT_TIME
cd $R
python3 tools/ct_summary.py gpurun_out/ct4 > gpurun_out/ct4_batch.txt; python3 tools/ct_summary.py gpurun_out/ct4pr > gpurun_out/ct4_perrec.txt
cat gpurun_out/ct4_batch.txt gpurun_out/ct4_perrec.txt | head -120
exit 0
  )
  ;;
ctlat)
  # per-record latency: default off / constant-time (old last step) / constant-time (tree), same box
  (
V=tools/variants
for run in "0 $V/lib_old.so" "1 $V/lib_old.so" "1 $V/lib_both.so" "0 $V/lib_both.so"; do set -- $run
  echo "== PTLS_MI355X_CONSTANT_TIME=$1 $2"
  PTLS_MI355X_CONSTANT_TIME=$1 timeout -k 10 120 python tools/latency.py $2 > gpurun_out/ctlat.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ctlat.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
ctpr)
  # round 3: constant-time evidence of the per-record path (picotls objects, CT by default) and its latency phases
  (
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
  )
  ;;
cttree)
  # constant-time tree A/B: parity of the CT paths, then default vs CT (old four-multiply last step, lane tree, lane tree +
  # combine tree) in one process per workload
  (
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ct.py tests/test_gpu_resources.py > gpurun_out/cttree_tests.log 2>&1
rc=$?; tail -3 gpurun_out/cttree_tests.log; [ $rc -ne 0 ] && exit $rc
V=tools/variants
for w in tls16k_1048576 quic1200_4194304 mixed_4194304; do set -- ${w/_/ }
  timeout -k 10 300 python tools/ab.py $V/lib_old.so $V/lib_old.so:ct $V/lib_tree.so:ct $V/lib_both.so:ct --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/cttree_$1.log 2>&1
  rc=$?; echo "== $1"; grep -v amdgpu.ids gpurun_out/cttree_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
deal)
  # chunk dealing (CHUNKS_PER_WG 0 = contiguous ranges, 4, 8, 16): GPU parity suite, then interleaved A/B at bench sizes
  (
bash tools/gpu_tests.sh || exit 1
V="tools/variants/lib_k0.so tools/variants/lib_k4.so tools/variants/lib_k8.so tools/variants/lib_k16.so"
for w in "mixedsorted 4194304" "tls16k 1048576" "quic1200 4194304" "mixed 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py $V --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$1.log | tail -8; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
early)
  # early GHASH tables (one-key launches): GPU suite, small-batch launches and per-record latency, noearly vs new
  (
bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python tools/small_batch.py tools/variants/lib_base.so tools/variants/lib_new.so > gpurun_out/small_batch.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/small_batch.log; [ $rc -ne 0 ] && exit $rc
LAT_BASE=tools/variants/noearly bash tools/gpu_lat_ab.sh
  )
  ;;
flags)
  # scheduler-flag sweep of the whole engine build (tools/ab.py, interleaved, identical output checked)
  (
V=tools/variants
L="$V/v0_base.so $V/v1_trackers.so $V/v2_nohighrp.so $V/v3_maxilp.so $V/v4_memclause.so $V/v5_minreg.so"
for w in tls16k_262144 quic1200_1048576 mixed_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 280 python tools/ab.py $L --workload $wl --records $n --rounds 3 --reps 2 > gpurun_out/flags_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/flags_$wl.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
full)
  # full measurement session: default bench (+e2e), the many-key config and the 32M x 1200 B config on one GPU
  (
timeout -k 10 600 python bench.py --e2e > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench default rc=$rc"; grep "^{" gpurun_out/bench_default.log | tail -1 | cut -c1-3000
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_default.log; exit $rc; }
timeout -k 10 600 python bench.py --workload mixed --extra= --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_mixed.log 2>&1
rc=$?; echo "bench mixed rc=$rc"; grep "^{" gpurun_out/bench_mixed.log | tail -1 | cut -c1-1500
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_mixed.log; exit $rc; }
timeout -k 10 600 python bench.py --workload mixedrand --extra= --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_mixedrand.log 2>&1
rc=$?; echo "bench mixedrand rc=$rc"; grep "^{" gpurun_out/bench_mixedrand.log | tail -1 | cut -c1-1500
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_mixedrand.log; exit $rc; }
timeout -k 10 600 python bench.py --workload shard1200 --extra= --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_shard.log 2>&1
rc=$?; echo "bench shard1200 rc=$rc"; grep "^{" gpurun_out/bench_shard.log | tail -1 | cut -c1-1500
exit $rc
  )
  ;;
hp)
  # round 3: header protection fused into the seal launch -- parity, batch cost, plain-seal A/B against the build before
  (
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lifecycle.py tests/test_gpu_resources.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
for r in 1 2; do
timeout -k 10 300 python tools/hp_cost.py --rounds 7 > gpurun_out/hp_cost_$r.txt 2>&1; rc=$?; echo "hp_cost rc=$rc"; grep hp_cost gpurun_out/hp_cost_$r.txt; [ $rc -ne 0 ] && exit $rc
done
for w in "quic1200 4194304" "tls16k 262144"; do
  set -- $w
  timeout -k 10 300 python tools/ab.py tools/variants/lib_prehp.so tools/variants/lib_hpfused.so --workload $1 --records $2 --rounds 5 > gpurun_out/ab_hp_$1.log 2>&1
  rc=$?; echo "ab $1 rc=$rc"; tail -2 gpurun_out/ab_hp_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
hpfuse)
  # fused per-record header protection: GPU suite, bulk A/B (previous build vs this one), per-record latency A/B
  (
bash tools/gpu_tests.sh || exit 1
V="tools/variants/lib_prev.so tools/variants/lib_new.so"
for w in "tls16k 1048576" "quic1200 4194304" "mixed 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py $V --workload $1 --records $2 --rounds 3 --reps 2 > gpurun_out/ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$1.log | tail -2; [ $rc -ne 0 ] && exit $rc
done
LAT_BASE=tools/variants/nofuse bash tools/gpu_lat_ab.sh
  )
  ;;
latbig)
  # long per-record calls (span path): wall times, then a kernel trace of the same
  (
timeout -k 10 120 python tools/lat_big.py 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/latbig; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o big -- python3 $GRAFT_REPO_ROOT/tools/lat_big.py > $OUT/log.txt 2>&1
rc=$?; echo rc=$rc; find $OUT -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150
exit $rc
  )
  ;;
latprof)
  # kernel trace of per-record seals (16 B, then 1200 B): the GPU time of a lone record's launch
  (
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/latprof; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o lat -- python3 $R/tools/lat_small.py > $OUT/log.txt 2>&1
rc=$?; echo rc=$rc; find $OUT -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
g = [r for r in rows if "gcm_chunked" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in g]
import statistics
for name, part in (("16 B", d[:300]), ("1200 B", d[300:600])):
    if part:
        print(name, "median kernel us", round(statistics.median(part), 2), "n", len(part))
PY
exit $rc
  )
  ;;
mixalign)
  # many-key mixed seal traffic attribution (tools/mixed_align.py): per layout a timing run, then one rocprofv3 --pmc
  # pass each for WRITE_SIZE and FETCH_SIZE (one TCC counter group per pass)
  (
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
  )
  ;;
mixalign2)
  # spill share of the many-key mixed seal traffic: the default and constant-time builds of the seal (113 vs 36 scratch
  # loads in the kernel's code) on the packed and line-aligned layouts: WRITE_SIZE, FETCH_SIZE and the VMEM instruction
  # counts, one rocprofv3 --pmc pass per process
  (
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for v in "packed " "packed --ct" "lines " "lines --ct"; do set -- $v; tag=$1${2:+_ct}
  for c in WRITE_SIZE FETCH_SIZE "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VMEM SQ_INSTS_FLAT"; do cn=${c%% *}
    timeout -k 10 150 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/mixalign2/${tag}_$cn -o p -- python3 $R/tools/mixed_align.py --layout $1 $2 --reps 2 > $R/gpurun_out/mixalign2_${tag}_$cn.log 2>&1
    rc=$?; echo "$tag $cn rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/mixalign2_${tag}_$cn.log; exit $rc; }
  done
done
exit 0
  )
  ;;
mixattr)
  # where the mixed-length many-key line loses against uniform records: the product build on AES-256
  # workloads of ~4 GiB payload: uniform 16 KiB, uniform 8 KiB (the mixed mean), mixed lengths under one key, and the
  # configs[3] batch itself (64K keys, full size so that every key has its 64 records)
  (
L=picotls_amd/_lib/libptls_mi355x.so
for w in tls16k256_262144 u8k256_524288 mixed1key_524288 mixed_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 200 python tools/ab.py $L --workload $wl --records $n --rounds 3 --reps 2 > gpurun_out/mixattr_$wl.log 2>&1
  rc=$?; echo "== $wl"; grep -v amdgpu.ids gpurun_out/mixattr_$wl.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
mt_stats)
  # combining statistics of the per-record path at 1, 4 and 16 threads, 1200-byte records, combine 0 / 1 / 2 / 4
  (
for C in 0 1 2 4; do
  for T in 1 4 16; do
    PTLS_MI355X_COMBINE_STATS=1 PTLS_MI355X_COMBINE=$C MT_THREADS=$T timeout -k 10 60 tools/_bin/mt_records 0.5 1200 > gpurun_out/mts.log 2>&1; rc=$?
    echo "== combine=$C threads=$T rc=$rc"; grep -v amdgpu.ids gpurun_out/mts.log | grep -E "threads +$T:|combine stats"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
  )
  ;;
phases)
  # phase breakdown of the chunked kernel (ENGINE_PROFILE build): a lone record, a 1000-record batch, the bench batches
  (
cd tools
for w in "tls16k 1" "tls16k 1000" "quic1200 1000" "tls16k 262144" "mixed 4194304" "mixed1key 1048576"; do set -- $w
  timeout -k 10 200 python prof_phases.py variants/lib_prof.so --workload $1 --records $2 --reps 5 2>&1 | grep -v amdgpu.ids || exit 1
done
exit 0
  )
  ;;
rank)
  # direct ranking of a small first run vs the bucket sort: small batches, bulk sanity, phases, GPU suite
  (
A=tools/variants/lib_copy.so; B=tools/variants/lib_rank.so
timeout -k 10 300 python tools/small_batch.py $A $B --rounds 5 > gpurun_out/rank_small.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/rank_small.log | cut -c1-130; [ $rc -ne 0 ] && exit $rc
for w in mixed_4194304 quic1200_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 280 python tools/ab.py $A $B --workload $wl --records $n --rounds 3 --reps 2 > gpurun_out/rank_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/rank_$wl.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 python tools/latency.py > gpurun_out/rank_lat.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/rank_lat.log; [ $rc -ne 0 ] && exit $rc
cd tools
for w in "tls16k 1000" "quic1200 1000"; do set -- $w
  timeout -k 10 200 python prof_phases.py variants/lib_prof.so --workload $1 --records $2 --reps 5 2>&1 | grep -v amdgpu.ids || exit 1
done
cd ..
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; exit $rc
  )
  ;;
round3)
  # round-3 check: every GPU test, the default bench line (all BASELINE configs incl. shard1200), HP batch cost, the small
  # batches with long records
  (
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -30; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { tail -80 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_default.log
[ $rc -ne 0 ] && { tail -30 gpurun_out/bench_default.err; exit $rc; }
timeout -k 10 300 python tools/hp_cost.py --rounds 7 > gpurun_out/hp_cost.txt 2>&1; rc=$?; grep hp_cost gpurun_out/hp_cost.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/small_batch.py --rounds 3 > gpurun_out/small_batch.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/small_batch.txt | head -8
exit $rc
  )
  ;;
spill_ab)
  # round 3: parity tests, then interleaved A/B of the spill reduction (lib_old = round 2, lib_new2 = now) on the BASELINE
  # shapes, then rocprofv3 kernel trace + PMC passes (seal and open) for tls16k, quic1200 and mixed with the new build
  (
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_ct.py tests/test_gpu_resources.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
for w in "tls16k 262144" "quic1200 2097152" "mixed 4194304"; do
  set -- $w
  timeout -k 10 300 python tools/ab.py tools/variants/lib_old.so tools/variants/lib_new2.so --workload $1 --records $2 --rounds 5 > gpurun_out/ab_spill_$1.log 2>&1
  rc=$?; echo "ab $1 rc=$rc"; tail -2 gpurun_out/ab_spill_$1.log; [ $rc -ne 0 ] && exit $rc
done
for w in "tls16k 262144" "quic1200 2097152" "mixed 1048576"; do
  set -- $w
  bash tools/gpu_prof.sh $1 $2 r3 > gpurun_out/prof_r3_$1.log 2>&1; rc=$?; echo "prof $1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
split)
  # first scan on wave 0 alone while waves 1-15 copy the AES tables, vs every wave copying first: small batches, bulk, phases, GPU suite
  (
A=tools/variants/lib_rank.so; B=tools/variants/lib_split.so
timeout -k 10 300 python tools/small_batch.py $A $B --rounds 5 > gpurun_out/split_small.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/split_small.log | cut -c1-130; [ $rc -ne 0 ] && exit $rc
for w in mixed_4194304 quic1200_4194304; do n=${w##*_}; wl=${w%_*}
  timeout -k 10 280 python tools/ab.py $A $B --workload $wl --records $n --rounds 3 --reps 2 > gpurun_out/split_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/split_$wl.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 python tools/latency.py > gpurun_out/split_lat.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/split_lat.log; [ $rc -ne 0 ] && exit $rc
cd tools
for w in "tls16k 1" "tls16k 1000" "quic1200 1000"; do set -- $w
  timeout -k 10 200 python prof_phases.py variants/lib_prof.so --workload $1 --records $2 --reps 5 2>&1 | grep -v amdgpu.ids || exit 1
done
cd ..
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; exit $rc
  )
  ;;
spread)
  # round 3: long records in small one-key batches over many workgroups (spread_pieces) -- parity, small-batch timing
  # against the build before, bulk A/B
  (
timeout -k 10 600 python -u -m pytest tests/test_gpu_lifecycle.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python tools/small_batch.py tools/variants/lib_prespread.so tools/variants/lib_spread.so --rounds 4 > gpurun_out/small_spread.txt 2>&1; rc=$?; echo "small rc=$rc"; grep -v amdgpu gpurun_out/small_spread.txt | tail -40; [ $rc -ne 0 ] && exit $rc
for w in "quic1200 4194304" "tls16k 262144" "mixed 4194304"; do
  set -- $w
  timeout -k 10 300 python tools/ab.py tools/variants/lib_prespread.so tools/variants/lib_spread.so --workload $1 --records $2 --rounds 4 > gpurun_out/ab_spread_$1.log 2>&1
  rc=$?; echo "ab $1 rc=$rc"; tail -2 gpurun_out/ab_spread_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
ttab)
  # AES table copy with 8 loads in flight per thread (vs 4): GPU suite, small-batch launches and per-record latency A/B,
  # bulk A/B
  (
bash tools/gpu_tests.sh -k "first_run or per_record or fuzz" || exit 1
timeout -k 10 300 python tools/small_batch.py tools/variants/lib_base.so tools/variants/lib_new.so > gpurun_out/small_batch.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/small_batch.log; [ $rc -ne 0 ] && exit $rc
for w in "tls16k 1048576" "quic1200 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py tools/variants/lib_base.so tools/variants/lib_new.so --workload $1 --records $2 --rounds 3 --reps 2 > gpurun_out/ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$1.log | tail -2; [ $rc -ne 0 ] && exit $rc
done
LAT_BASE=tools/variants/b4 LAT_NEW=tools/variants/b8 bash tools/gpu_lat_ab.sh
  )
  ;;
ab_three)
  # interleaved A/B of tools/variants/*.so on tls16k, quic1200 and the 64K-key mixed config at full size
  (
for w in ${AB_WORKLOADS:-tls16k_1048576 quic1200_4194304 mixed_4194304}; do set -- ${w/_/ }
timeout -k 10 300 python tools/ab.py tools/variants/*.so --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/ab_$1.log 2>&1
rc=$?; echo "== $1"; grep -v amdgpu.ids gpurun_out/ab_$1.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
  )
  ;;
sched)
  # one engine build, every analysis workload under both schedules (1 = lockstep, 2 = chunked)
  (
for spec in "tls16k 262144 1" "tls16k 262144 2" "quic1200 1048576 1" "quic1200 1048576 2" "mixed1key 1048576 2" "mixed 4194304 2"; do
  set -- $spec
  echo "== $1 n=$2 schedule=$3"
  timeout -k 10 300 python tools/ab.py tools/variants/*.so --workload $1 --records $2 --schedule $3 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
done
  )
  ;;
*)
  echo "usage: bash tools/gpu_recipes.sh <recipe>; recipes:"; grep -E "^[a-z0-9_]+\)$" "$0" | tr -d ")"; exit 2 ;;
esac
