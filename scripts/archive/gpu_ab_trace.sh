# Rollout A/B + 8-wave phase trace: policy / rollout tests, ab_rollout.py over the builds in $BUILDS
# (in-tree "base" first), then the k_rollout_steps stamps of all 8 waves (scripts/trace8, make TRACE=1
# TRACE_WAVES=8).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${PYTEST_SEL:-tests/test_gpu_policy_gae.py} -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_ab.log; grep -E "^E  |FAILED" gpurun_out/pytest_ab.log | head -20
[ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-3} timeout -k 10 900 python scripts/ab_rollout.py base ${BUILDS} || exit 1
if [ -d scripts/trace8 ]; then
  UAVHIP_LIB=$PWD/scripts/trace8/libuavhip.so WAVES=8 STEPS=1 timeout -k 10 120 python scripts/policy_trace.py > gpurun_out/trace8.txt 2>&1 || { tail -5 gpurun_out/trace8.txt; exit 1; }
  cat gpurun_out/trace8.txt
fi
