set +e
cd $GRAFT_REPO_ROOT
# one engine build, every analysis workload under both schedules (1 = lockstep, 2 = chunked)
for spec in "tls16k 262144 1" "tls16k 262144 2" "quic1200 1048576 1" "quic1200 1048576 2" "mixed1key 1048576 2" "mixed 4194304 2"; do
  set -- $spec
  echo "== $1 n=$2 schedule=$3"
  timeout -k 10 300 python tools/ab.py tools/variants/*.so --workload $1 --records $2 --schedule $3 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
done
