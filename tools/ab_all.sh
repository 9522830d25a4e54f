# interleaved A/B of tools/variants/*.so on the three single-GPU configs (AUTO schedule)
set +e
cd $GRAFT_REPO_ROOT
for spec in "tls16k 262144" "quic1200 1048576" "mixed 1048576"; do
  set -- $spec
  echo "== $1 n=$2"
  timeout -k 10 300 python tools/ab.py tools/variants/*.so --workload $1 --records $2 --rounds 4 2>&1 | grep -v amdgpu.ids || exit 1
done
