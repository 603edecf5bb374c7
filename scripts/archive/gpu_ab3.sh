# Policy + training tests, rollout A/B (base vs $RBUILDS), training per-kernel A/B (base vs $TBUILDS)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${PYTEST_SEL:-tests/test_gpu_policy_gae.py tests/test_gpu_train.py} -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_ab3.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_ab3.log; grep -E "^E  |FAILED" gpurun_out/pytest_ab3.log | head -20
[ $rc -eq 0 ] || exit $rc
if [ -n "$RBUILDS" ]; then ROUNDS=${ROUNDS:-3} timeout -k 10 900 python scripts/ab_rollout.py base $RBUILDS || exit 1; fi
if [ -n "$TBUILDS" ]; then
  BS=4096 N=65536 MAXSTEPS=16 bash scripts/ab_kstats.sh base $TBUILDS base $TBUILDS 2>&1 | grep -E "==|backward" || exit 1
  for b in base $TBUILDS; do python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/ab_$b/run_kernel_stats.csv')):
    if 'forward' in r['Name']: print('$b forward', round(float(r['AverageNs'])/1000,2))"; done
fi
if [ -n "$T64BUILDS" ]; then
  bash scripts/ab_kstats.sh base $T64BUILDS base $T64BUILDS 2>&1 | grep -E "==" || exit 1
fi
