# Round-4 call s: per-problem chunk lengths in the chunked weight-gradient schedule (three-plane key-row
# problems get UAVHIP_WGRAD_P3_RATIO x the two-plane chunk) -- parity tests, then k_wgrad times per ratio.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_policy_gae.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_r04s.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed|worst bar|replay" gpurun_out/pytest_r04s.log | tail -8; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for m in 1.0 0.75 0.6; do echo -n "ratio=$m: "; UAVHIP_WGRAD_P3_RATIO=$m KERNELS="k_wgrad" TAG=r04s_${m}_$r bash scripts/ab_kernel_time.sh base || exit 1; done; done
echo all done
