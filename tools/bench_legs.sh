#!/bin/bash
# the default bench line on the box, timed, with a per-leg summary: bash tools/bench_legs.sh <tag>
set +e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-b}; mkdir -p gpurun_out
t0=$(date +%s)
timeout -k 10 700 python bench.py > gpurun_out/${tag}.json 2> gpurun_out/${tag}.err; rc=$?
echo "bench rc=$rc, $(( $(date +%s) - t0 )) s"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${tag}.err; exit $rc; }
tail -1 gpurun_out/${tag}.json | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('value', d['value'], 'frac', d['roofline']['frac'], 'seal', d['seal_GiBps'], 'open', d['open_GiBps'])
for k, v in d['extra'].items():
    print(k, v['value'], v.get('seal_GiBps'), v.get('open_GiBps'), v.get('verified'))
"
