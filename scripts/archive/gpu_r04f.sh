# Round-4 call f: policy / rollout tests after the NaN-preserving ReLU, then a same-box A/B of the
# rollout: current build, with a per-element overflow guard in the plane writers (EXP=41 at the time;
# since dropped), without the delta env stores (EXP=42),
# and round 3's final code (scripts/r03: bash scripts/build_variant.sh r03 407cce9).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_policy_gae.py tests/test_gpu_env.py tests/test_gpu_train.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_r04f.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_r04f.log | tail -4; [ $rc -le 1 ] || exit $rc
ROUNDS=3 timeout -k 10 900 python scripts/ab_rollout.py base noguard nodelta r03 > gpurun_out/ab_r04f.txt 2>&1 || { tail -20 gpurun_out/ab_r04f.txt; exit 1; }
cat gpurun_out/ab_r04f.txt
