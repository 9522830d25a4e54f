#!/bin/bash
# Round-5 GPU recipes (run on the GPU box through gpurun, from the repository root):  bash tools/gpu_r5.sh <name>
# Variant engines for these recipes live under tools/gv/<name>/libptls_mi355x.so (built with tools/mkvariant.sh-style
# hipcc lines; tools/gv is not in .gpurunignore, unlike tools/variants).
set +e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
recipe=$1; shift
case "$recipe" in
check)
  # the round's new and changed GPU tests: exact-shape headline parity (EXT 3 counted), W8 pairs on streams and threads
  # at whole-run sizes, the handled-error regression test, the lockstep / constant-time rule, the bench launch tests
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_headline.py \
      tests/test_gpu_w8.py tests/test_gpu_resources.py tests/test_gpu_bench_launch.py \
      "tests/test_gpu_parity.py::test_picotls_vtable_tls12_with_handled_errors_left_on_the_thread" \
      > gpurun_out/r5_check.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r5_check.log | tail -40; tail -3 gpurun_out/r5_check.log
  exit $rc
  ;;
lasterr5)
  # the regression test against an engine with LAUNCH_CLEAR() compiled out (must fail the
  # TLS 1.2 checks) and against the shipped engine (must pass); the C binary is the same
  {
  echo "== engine built with -DLAUNCH_CLEAR_NOOP=1 (tools/gv/noop)"
  LD_LIBRARY_PATH=$PWD/tools/gv/noop timeout -k 10 120 tests/c/_bin/test_vtable lasterr; echo "exit status $?"
  echo "== shipped engine (picotls_amd/_lib)"
  timeout -k 10 120 tests/c/_bin/test_vtable lasterr; echo "exit status $?"
  } > gpurun_out/lasterr_regression.txt 2>&1
  cat gpurun_out/lasterr_regression.txt | tail -40
  grep -q "== shipped" gpurun_out/lasterr_regression.txt && tail -1 gpurun_out/lasterr_regression.txt | grep -q "exit status 0"
  ;;
firstcall)
  # the TLS 1.2 first-call tag difference of lasterr5 (round 5): fresh processes with and without the injected error,
  # the shipped engine and the base variant, then the whole vtable suite
  for v in shipped base; do for inj in 1 0; do
    if [ $v = base ]; then LIB="LD_LIBRARY_PATH=$PWD/tools/gv/base"; else LIB=""; fi
    if [ $inj = 0 ]; then NI="PTLS_TEST_NO_INJECT=1"; else NI=""; fi
    for rep in 1 2; do
      env $LIB $NI timeout -k 10 120 tests/c/_bin/test_vtable lasterr > gpurun_out/fc_${v}_inj${inj}_$rep.txt 2>&1; rc=$?
      echo "== $v inject=$inj rep=$rep exit=$rc: $(grep -c '^not ok' gpurun_out/fc_${v}_inj${inj}_$rep.txt) failed checks"
      grep -A2 "^not ok" gpurun_out/fc_${v}_inj${inj}_$rep.txt | head -8
      [ $rc -gt 1 ] && exit $rc
    done
  done; done
  timeout -k 10 300 tests/c/_bin/test_vtable > gpurun_out/fc_full.txt 2>&1; rc=$?
  echo "== full suite exit=$rc"; grep "^not ok" gpurun_out/fc_full.txt | head; tail -2 gpurun_out/fc_full.txt
  exit 0
  ;;
firstcall2)
  # (round 5) fresh processes whose first engine calls are picotls' TLS 1.2 exchanges (test_vtable lasterr): how often the
  # first record's tag differs, what the wrong tag holds, and (PTLS_MI355X_DIAG=1) whether result bytes changed after the
  # completion words were seen
  nf=0
  for i in $(seq 1 ${1:-16}); do for d in 1 0; do
    PTLS_MI355X_DIAG=$d timeout -k 10 60 tests/c/_bin/test_vtable lasterr > gpurun_out/fc2_${i}_d$d.txt 2>&1; rc=$?
    [ $rc -gt 1 ] && { echo "process $i diag=$d exit $rc"; tail -5 gpurun_out/fc2_${i}_d$d.txt; exit $rc; }
    if [ $rc -ne 0 ] || grep -q "ptls_mi355x diag" gpurun_out/fc2_${i}_d$d.txt; then
      nf=$((nf+1)); echo "== process $i diag=$d exit $rc"; grep -E "^not ok|^#|diag" gpurun_out/fc2_${i}_d$d.txt | head -12
    fi
  done; done
  echo "processes with a difference: $nf of $((2 * ${1:-16}))"
  exit 0
  ;;
ct6)
  # (round 5) LDS bank conflicts of the many-key mixed kernel per dispatch (rocprofv3 --pmc
  # SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS, one process per case, 2 seals + 2 opens): the product build over 4 keys x 3
  # payloads and a length-permuted batch; the CT_PROBE_CONST diagnosis build (tools/gv/ctconst: every data-derived LDS
  # address replaced by a constant) on the same batch
  (
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
run() {  # name, extra args
  timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/ct6/$1 -o p -- python3 $R/tools/ct_probe.py --workload mixed --records 4194304 --reps 2 ${@:2} > $R/gpurun_out/ct6_$1.log 2>&1
  rc=$?; echo "$1 rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/ct6_$1.log; exit $rc; }
}
for k in 1 2 3 4; do for pl in zero random ones; do run k${k}_$pl --key-seed $k --payload $pl; done; done
run k1_random_permuted --key-seed 1 --payload random --permute 7
run ctconst_k1_random --key-seed 1 --payload random --lib $R/tools/gv/ctconst/libptls_mi355x.so --no-check
run ctconst_k2_zero --key-seed 2 --payload zero --lib $R/tools/gv/ctconst/libptls_mi355x.so --no-check
cd $R
python3 tools/ct_summary.py gpurun_out/ct6 > gpurun_out/ct6_mixed.txt; cat gpurun_out/ct6_mixed.txt
exit 0
  )
  ;;
ctsite)
  # (round 5) which batch property the many-key mixed kernel's conflict cycles follow: the same length mix under one
  # key and under 64K keys, uniform lengths under 64K keys, and the sorted mix (rocprofv3 --pmc, 2 seals + 2 opens)
  (
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
run() {  # name, extra args
  timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/ctsite/$1 -o p -- python3 $R/tools/ct_probe.py --records 4194304 --reps 2 ${@:2} > $R/gpurun_out/ctsite_$1.log 2>&1
  rc=$?; echo "$1 rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/ctsite_$1.log; exit $rc; }
}
run mixed_1key --workload mixed --keys 1
run mixed_64k --workload mixed
run mixed_4k --workload mixed --keys 4096
run quic1200_64k --workload quic1200 --keys 65536
run u8k_64k --workload u8k256 --keys 65536
run mixedsorted_1key --workload mixedsorted
cd $R
python3 tools/ct_summary.py gpurun_out/ctsite > gpurun_out/ctsite.txt; cat gpurun_out/ctsite.txt
exit 0
  )
  ;;
ab)
  # interleaved A/B (tools/ab.py, one process per workload) of tools/gv/<name> engines at the full BASELINE sizes:
  #   bash tools/gpu_r5.sh ab "base scat" [tag] [workloads...]
  names=$1; tag=${2:-ab}; shift 2 2>/dev/null
  wls=${*:-"quic1200:4194304 tls16k:1048576 mixed:4194304"}
  libs=""; for n in $names; do libs="$libs tools/gv/$n/libptls_mi355x.so"; done
  for wn in $wls; do w=${wn%%:*}; r=${wn##*:}
    timeout -k 10 400 python tools/ab.py $libs --workload $w --records $r --rounds 5 --reps 2 > gpurun_out/${tag}_$w.log 2>&1
    rc=$?; echo "== $w rc=$rc"; grep -v amdgpu.ids gpurun_out/${tag}_$w.log | tail -6; [ $rc -ne 0 ] && exit $rc
  done
  exit 0
  ;;
wcal)
  # (round 5) WRITE_SIZE / FETCH_SIZE against known byte counts for the engine's access shapes (tools/mb/wcal.hip):
  # wave-wide 16 B per lane, 128-byte lines per 8-lane group, 64-byte half lines per quad; 1M packed 1216-byte records
  # (the QUIC batch's sealed records) and 1280-byte ones (line multiples), with and without work between steps
  (
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
run() {  # name, counter, wcal args
  timeout -k 10 120 rocprofv3 --pmc $2 --output-format csv -d $R/gpurun_out/wcal/$1 -o p -- $R/tools/mb/wcal.bin ${@:3} > $R/gpurun_out/wcal/$1.log 2>&1
  rc=$?; echo "$1 rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/wcal/$1.log; exit $rc; }
}
mkdir -p $R/gpurun_out/wcal
if [ "$1" = 2 ]; then  # (second pass: non-temporal and paired halves, longer gaps; the TCC request counters)
  timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/wcal/counters_avail.txt 2>&1
  for m in 1 2 3 4; do for sp in 200 2000; do
    run st_m${m}_1216_s$sp WRITE_SIZE $m 0 1048576 1216 $sp 2
    run ld_m${m}_1216_s$sp FETCH_SIZE $m 1 1048576 1216 $sp 2
  done; done
else
for m in 0 1 2; do for sp in 0 200; do
  run st_m${m}_1216_s$sp WRITE_SIZE $m 0 1048576 1216 $sp 3
  run ld_m${m}_1216_s$sp FETCH_SIZE $m 1 1048576 1216 $sp 3
done; done
run st_m2_1280_s200 WRITE_SIZE 2 0 1048576 1280 200 3
run ld_m2_1280_s200 FETCH_SIZE 2 1 1048576 1280 200 3
fi
cd $R
python3 tools/wcal_summary.py gpurun_out/wcal > gpurun_out/wcal$1.txt; cat gpurun_out/wcal$1.txt; grep -E "TCC_EA0_(RD|WR)REQ" gpurun_out/wcal/counters_avail.txt | head -20
exit 0
  )
  ;;
wpmc)
  # (round 5) WRITE_SIZE and FETCH_SIZE of one workload's seal/open launches per engine variant (tools/gv/<name>):
  #   bash tools/gpu_r5.sh wpmc "base pair" quic1200 4194304
  (
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/wpmc
for n in $1; do for c in WRITE_SIZE FETCH_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/wpmc/${n}_$c -o p -- python3 $R/tools/ab.py $R/tools/gv/$n/libptls_mi355x.so --workload $2 --records $3 --rounds 1 --reps 1 > $R/gpurun_out/wpmc/${n}_$c.log 2>&1
  rc=$?; echo "$n $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/wpmc/${n}_$c.log; exit $rc; }
done; done
cd $R; python3 tools/wpmc_summary.py gpurun_out/wpmc $2 $3 > gpurun_out/wpmc_$2.txt; cat gpurun_out/wpmc_$2.txt
exit 0
  )
  ;;
*)
  echo "unknown recipe $recipe"; exit 2 ;;
esac
