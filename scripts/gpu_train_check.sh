# Training-step check: the -m gpu training / policy tests, then per-kernel averages at minibatch 64 and 4096.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dropin.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_train.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_train.log | tail -40
[ $rc -le 1 ] || exit $rc
bash scripts/ab_kstats.sh base ${BUILDS} || exit 1
BS=4096 N=65536 MAXSTEPS=16 bash scripts/ab_kstats.sh base || exit 1
exit $rc
