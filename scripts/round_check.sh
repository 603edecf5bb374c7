#!/bin/bash
# tests + smoke + default bench + rollout / training profiles (each GPU step under its own timeout)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
TAG=r01 timeout -k 10 900 bash scripts/profile.sh || exit $?
TAG=r01 timeout -k 10 900 bash scripts/profile_train.sh || exit $?
echo ALLDONE > gpurun_out/round.done
