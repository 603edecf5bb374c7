# Round-4 call aa: GAE staging loads batched and k_adv_normalize's loads ahead of its statistics
# (this tree vs scripts/r04z_head = HEAD); the position-split backward's both-chunk attention loads
# (scripts/r04z_head vs scripts/r04z_noattn = HEAD with that change reverted). -m gpu first.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r04aa.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_r04aa.log | tail -12
[ $rc -le 1 ] || { tail -40 gpurun_out/pytest_r04aa.log; exit $rc; }
for r in 1 2; do
  for b in r04z_head base; do
    KERNELS="k_gae k_adv_normalize k_policy_rows_fill k_policy_forward" TAG=r04aa_$r bash scripts/ab_rollout_kernels.sh $b || exit 1
  done
done
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for b in r04z_noattn r04z_head; do
    BS=64 MAXSTEPS=256 N=16384 KERNELS="k_ps_b1 k_ps_b2 k_ps_b3" TAG=r04aa_$r bash scripts/ab_kernel_time.sh $b || exit 1
  done
done
echo all done
