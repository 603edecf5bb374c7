# Same-box A/B of rollout builds (scripts/ab_rollout.py, AB="base v_x ...") and phase traces of TRACE
# builds (TRACES="t_x ..."); optionally a pytest subset first (PYTEST_K).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-abt}
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_$TAG.log | tail -15
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "$AB" ]; then
  ROUNDS=${ROUNDS:-3} timeout -k 10 900 python -u scripts/ab_rollout.py $AB > gpurun_out/ab_$TAG.txt 2>&1 || { tail -20 gpurun_out/ab_$TAG.txt; exit 1; }
  tail -4 gpurun_out/ab_$TAG.txt
fi
for b in $TRACES; do
  UAVHIP_ACCEPT_PREV_ABI=1 UAVHIP_LIB=$PWD/scripts/$b/libuavhip.so STEPS=1 timeout -k 10 180 python scripts/policy_trace.py > gpurun_out/trace_${TAG}_$b.log 2>&1 || { tail -20 gpurun_out/trace_${TAG}_$b.log; exit 1; }
  echo "== $b"; tail -3 gpurun_out/trace_${TAG}_$b.log | head -1
done
