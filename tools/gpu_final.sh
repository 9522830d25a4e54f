#!/bin/bash
# The round's end-to-end GPU check (bounded steps, chained): the -m gpu suite, smoke(), the default bench line.
#   bash tools/gpu_final.sh <tag>     -> gpurun_out/<tag>_pytest.log, <tag>_smoke.log, <tag>_bench.json / .err
set +e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-final}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/${tag}_pytest.log | head -20; tail -2 gpurun_out/${tag}_pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1; src=$?
echo "smoke rc=$src"; tail -1 gpurun_out/${tag}_smoke.log; [ $src -ne 0 ] && exit $src
timeout -k 10 600 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err; brc=$?
echo "bench rc=$brc"; python -c "
import json,sys
d=json.loads(open('gpurun_out/${tag}_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'verified', d['verified'])
for k,v in d.get('extra',{}).items(): print(k, v['value'], v.get('seal_hbm_frac'), v['verified'])
" ; exit $(( rc | brc ))
