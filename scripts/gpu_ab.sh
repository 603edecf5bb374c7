# -m gpu (or PYTEST_K) then a same-box A/B of rollout builds (scripts/ab_rollout.py; AB="base v_x ...").
#   TAG=r05d AB="base v_rng v_r4" bash scripts/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ -z "$SKIP_TESTS" ]; then
  K=${PYTEST_K:+-k "$PYTEST_K"}
  eval timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread $K > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_$TAG.log | tail -15
  [ $rc -le 1 ] || { tail -40 gpurun_out/pytest_$TAG.log; exit $rc; }
fi
ROUNDS=${ROUNDS:-3} timeout -k 10 900 python -u scripts/ab_rollout.py ${AB:-base} > gpurun_out/ab_$TAG.txt 2>&1 || { tail -20 gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
