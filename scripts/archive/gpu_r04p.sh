# Round-4 call p: two-plane weight-gradient tiles except the key rows -- the training parity tests,
# then k_wgrad times three-plane everywhere (UAVHIP_WGRAD_PLANES=3) vs the default, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_policy_gae.py tests/test_gpu_dropin.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_r04p.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed|worst bar|replay" gpurun_out/pytest_r04p.log | tail -12; [ $rc -le 1 ] || exit $rc
for r in 1 2 3; do for m in 3 2; do echo -n "planes=$m: "; UAVHIP_WGRAD_PLANES=$m KERNELS="k_wgrad k_policy_backward" TAG=r04p_${m}_$r bash scripts/ab_kernel_time.sh base || exit 1; done; done
for r in 1 2 3; do for m in 3 2; do echo -n "planes=$m mb64: "; UAVHIP_WGRAD_PLANES=$m KERNELS="k_wgrad" BS=64 N=16384 MAXSTEPS=256 TAG=r04p64_${m}_$r bash scripts/ab_kernel_time.sh base || exit 1; done; done
echo all done
