# Round-4 calls x / y (RTAG=r04y): the ring fill (k_policy_rows_fill) with every operand issued ahead and
# (y) the Win pos_s table spread over six fill blocks; the position-split kernels with their operands
# issued ahead: -m gpu, then same-box A/Bs against the HEAD build (scripts/r04w_head).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${RTAG:-r04x}.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_${RTAG:-r04x}.log | tail -12
[ $rc -le 1 ] || { tail -40 gpurun_out/pytest_${RTAG:-r04x}.log; exit $rc; }
for r in 1 2 3; do
  for b in r04w_head base; do
    KERNELS="k_policy_rows_fill k_rollout_steps k_gae" TAG=${RTAG:-r04x}_$r bash scripts/ab_rollout_kernels.sh $b || exit 1
  done
done
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for b in r04w_head base; do
    BS=64 MAXSTEPS=256 N=16384 KERNELS="k_ps_f1 k_ps_f2 k_ps_f3 k_ps_b1 k_ps_b2 k_ps_b3" \
      TAG=${RTAG:-r04x}_$r bash scripts/ab_kernel_time.sh $b || exit 1
  done
done
echo all done
