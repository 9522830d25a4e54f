# quick A/B: parity subset + short bench on both headline sizes (no cpu baseline)
set +e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_quick.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --records ${1:-262144} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"
python - <<'PY'
import json
l=[x for x in open('gpurun_out/bench_quick.log') if x.startswith('{')]
d=json.loads(l[-1])
print('tls16k', d['value'], 'seal', d['seal_GiBps'], 'open', d['open_GiBps'], 'frac', d['roofline']['frac'], d['verified'])
for k,v in d.get('extra',{}).items(): print(k, v['value'], 'seal', v['seal_GiBps'], 'open', v['open_GiBps'], v['verified'])
PY
exit $rc
