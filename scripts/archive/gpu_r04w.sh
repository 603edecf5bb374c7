# Round-4 call w: the position-split (minibatch <= 256) kernels with their global operands issued
# ahead (k_ps_f1..b3): the -m gpu suite, then a same-box A/B against the HEAD build
# (scripts/r04w_head, bash scripts/build_variant.sh r04w_head HEAD): per-kernel rocprofv3 averages at
# minibatch 64 and the update step time (train_probe.py), alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r04w.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_r04w.log | tail -12
[ $rc -le 1 ] || { tail -40 gpurun_out/pytest_r04w.log; exit $rc; }
for r in 1 2 3; do
  for b in r04w_head base; do
    BS=64 MAXSTEPS=256 N=16384 KERNELS="k_ps_f1 k_ps_f2 k_ps_f3 k_ps_b1 k_ps_b2 k_ps_b3 k_wgrad k_reduce_grads k_adam" \
      TAG=r04w_$r bash scripts/ab_kernel_time.sh $b || exit 1
  done
done
cd $GRAFT_REPO_ROOT
bash scripts/ab_train_quick.sh r04w_head base || exit 1
echo all done
