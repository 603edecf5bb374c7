# Round-4 call c: the env-step attribution with the realistic NOENV build (next windows still
# written) and the hot-ring build (EXP=32), the changed tests, then the full bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_policy_gae.py -m gpu -v -s --timeout 200 --timeout-method thread -k "overflow or large_activations or direct_mode" > gpurun_out/pytest_r04c.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_r04c.log | tail -1; [ $rc -le 1 ] || exit $rc
TAG=r04c bash scripts/profile_env_attrib.sh || exit 1
echo attrib ok
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python bench.py > gpurun_out/bench_r04c.json 2> gpurun_out/bench_r04c.err || { tail -20 gpurun_out/bench_r04c.err; exit 1; }
echo bench ok
