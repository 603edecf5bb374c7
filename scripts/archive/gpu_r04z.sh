# Round-4 call z: the rollout's bootstrap V(s_T) as a critic-only launch (uavhip_policy_value_rows):
# -m gpu, then same-box A/Bs of UAVHIP_BOOTSTRAP_FULL=1 (the full forward, as before) against the
# default: rocprofv3 kernel averages of a bare rollout, and the bench's rollout line, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r04z.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_r04z.log | tail -12
[ $rc -le 1 ] || { tail -40 gpurun_out/pytest_r04z.log; exit $rc; }
for r in 1 2; do
  for full in 1 0; do
    echo -n "bootstrap_full=$full "
    UAVHIP_BOOTSTRAP_FULL=$full KERNELS="k_policy_rows_fill k_rollout_steps k_policy_forward k_gae" TAG=r04z_${full}_$r \
      bash scripts/ab_rollout_kernels.sh base || exit 1
  done
done
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for full in 1 0; do
    echo -n "bootstrap_full=$full "
    UAVHIP_BOOTSTRAP_FULL=$full ROUNDS=1 timeout -k 10 300 python scripts/ab_rollout.py base | grep round || exit 1
  done
done
echo all done
