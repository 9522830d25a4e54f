# unit combine gmul_group (default) vs gmul_tab: interleaved A/B, then LDS bank conflicts of each on the mixed seal
set +e
cd $GRAFT_REPO_ROOT
V="tools/variants/lib_group.so tools/variants/lib_tab.so"
for w in "mixed 4194304" "mixedrand 4194304" "quic1200 4194304" "mixedsorted 4194304"; do set -- $w
  timeout -k 10 300 python tools/ab.py $V --workload $1 --records $2 --rounds 4 --reps 2 > gpurun_out/ab_$1.log 2>&1; rc=$?
  echo "== $1 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$1.log | tail -3; [ $rc -ne 0 ] && exit $rc
done
exit 0
