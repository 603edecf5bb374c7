# Full -m gpu suite, then the round-3 measurement set (gpu_r03c.sh) and the env-share PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_full.log | tail -3; grep -E "FAILED|^E  " gpurun_out/pytest_full.log | head -20
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r03d} bash scripts/gpu_r03c.sh || exit 1
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03d} bash scripts/profile_env_share.sh || exit 1
echo all done
