# Quick GPU check: an optional probe script, then a pytest selection (PYTEST_SEL).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "${PROBE}" ]; then timeout -k 10 240 python ${PROBE} > gpurun_out/probe.log 2>&1; rc=$?; cat gpurun_out/probe.log | tail -20; [ $rc -eq 0 ] || exit $rc; fi
timeout -k 10 900 python -u -m pytest ${PYTEST_SEL} -m gpu -v --maxfail=8 --timeout 400 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_sel.log | tail -40
exit $rc
