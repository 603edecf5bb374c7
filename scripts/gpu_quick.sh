# Quick GPU check after a kernel change: the -m gpu suite (or PYTEST_K), smoke, then a short bench line
# (no PPO / e2e / dropin / CPU legs unless BENCH_ARGS says otherwise).
#   TAG=r05x PYTEST_K="range or fp64" bash scripts/gpu_quick.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-quick}
K=${PYTEST_K:+-k "$PYTEST_K"}
eval timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread $K > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_$TAG.log | tail -15
[ $rc -le 1 ] || { tail -40 gpurun_out/pytest_$TAG.log; exit $rc; }
timeout -k 10 600 python bench.py ${BENCH_ARGS:---no-ppo --no-e2e --no-dropin --no-cpu-baseline --no-env-fused} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]); r=d['roofline']
print('value', d['value'], 'kernel ms/step', r['avg_launch_ms'], 'frac', r['frac'])
e=d.get('env_roofline') or {}; print('env', e.get('avg_launch_ms'), (e.get('differential') or {}).get('product_vs_headline'))
"
exit $rc
