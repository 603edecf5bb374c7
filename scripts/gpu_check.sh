#!/bin/bash
# GPU-box check: smoke, then the gpu test suite, then a short bench. Each step has its own time
# limit; a crash-class exit (abort/segfault/timeout/kill) stops the script before the next GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
ok() { case "$1" in 0|1|2|5) return 0;; *) return 1;; esac; }   # 0 ok, 1/2/5 = python/pytest failures
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/smoke.log; ok $rc || exit $rc
KARGS=(); [ -n "$PYTEST_K" ] && KARGS=(-k "$PYTEST_K")
timeout -k 10 700 python -m pytest tests -m gpu -q --timeout=300 -p no:cacheprovider "${KARGS[@]}" > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/pytest.log; ok $rc || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py $BENCH > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/bench.log; exit $rc
fi
