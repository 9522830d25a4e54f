# rocprofv3 summaries of the three bench workloads at bench sizes (see tools/gpu_prof.sh); stop at the first failure
set +e
cd $GRAFT_REPO_ROOT
for w in "tls16k 1048576" "quic1200 4194304" "mixed 4194304"; do set -- $w
  bash tools/gpu_prof.sh $1 $2 ${PROF_TAG:-r2f} || exit 1
done
exit 0
