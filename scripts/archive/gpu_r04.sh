# Round-4 measurement call: the -m gpu suite, smoke, the full bench line, then the profiles the bench
# line reads (profile.sh: k_rollout_steps kernel stats + FETCH / WRITE PMC; profile_env_counters.sh:
# the env-only kernels' counters; profile_env_share.sh: product vs NOENV build). Every GPU step under
# its own time limit; the call stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04a}
if [ -z "$SKIP_TESTS" ]; then
  # assertion failures (rc 1) are read afterwards and the measurements still run; a crash, abort or
  # time limit (any other rc) ends the call
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_$TAG.log | tail -12
  [ $rc -le 1 ] || { tail -40 gpurun_out/pytest_$TAG.log; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
  echo smoke ok
fi
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo bench ok
[ -n "$SKIP_PROFILES" ] && exit 0
TAG=$TAG bash scripts/profile.sh || exit 1
echo profile ok
cd $GRAFT_REPO_ROOT
TAG=$TAG bash scripts/profile_env_counters.sh || exit 1
echo env counters ok
cd $GRAFT_REPO_ROOT
TAG=$TAG bash scripts/profile_env_share.sh || exit 1
echo all done
