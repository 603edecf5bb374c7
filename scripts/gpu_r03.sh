# Round-3 GPU session: -m gpu suite, smoke, env-share probe, bench, env-share profile.
# pytest failures (exit 1) do not stop the later steps; a timeout / crash / fault does.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=6 --timeout 400 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_full.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_full.log
[ $rc -le 1 ] || exit $rc
if [ -n "${ONLY_TESTS}" ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python scripts/env_phase.py > gpurun_out/env_phase.json 2> gpurun_out/env_phase.err || { tail -5 gpurun_out/env_phase.err; exit 1; }
cat gpurun_out/env_phase.json
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
if [ -n "${ENVSHARE}" ]; then TAG=r03 timeout -k 10 900 bash scripts/profile_env_share.sh || exit 1; fi
exit $rc
