# Quick GPU check: a pytest selection (PYTEST_SEL, -m gpu) then the bench (no CPU baseline legs).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${PYTEST_SEL} -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_sel.log | tail -40
grep -E "^E  " gpurun_out/pytest_sel.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail -20 gpurun_out/bench_q.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_q.json'))
r=d['roofline']; print('value %.3e  ms/step %.3f  k_rollout_steps %.2f us/step  frac %.3f exec %.3f' % (d['value'], d['ms_per_step'], r['avg_launch_ms']*1e3, r['frac'], r['executed_frac']))
p=d.get('ppo_samples_per_s'); m=d.get('ppo_samples_per_s_mb64')
print('ppo', p and p['value'], 'mb64', m and m['value'], m and m.get('ms_per_optimizer_step'))
"
exit $rc
