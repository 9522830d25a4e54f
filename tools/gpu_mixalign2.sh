# spill share of the many-key mixed seal traffic: the default and constant-time builds of the seal (113 vs 36 scratch
# loads in the kernel's code) on the packed and line-aligned layouts: WRITE_SIZE, FETCH_SIZE and the VMEM instruction
# counts, one rocprofv3 --pmc pass per process
set +e
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for v in "packed " "packed --ct" "lines " "lines --ct"; do set -- $v; tag=$1${2:+_ct}
  for c in WRITE_SIZE FETCH_SIZE "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VMEM SQ_INSTS_FLAT"; do cn=${c%% *}
    timeout -k 10 150 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/mixalign2/${tag}_$cn -o p -- python3 $R/tools/mixed_align.py --layout $1 $2 --reps 2 > $R/gpurun_out/mixalign2_${tag}_$cn.log 2>&1
    rc=$?; echo "$tag $cn rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/mixalign2_${tag}_$cn.log; exit $rc; }
  done
done
exit 0
