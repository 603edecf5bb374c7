# Round-4 call ab: k_reduce_grads' tile mode with 16 part groups per block (this tree) against HEAD
# (scripts/r04ab_head): -m gpu, then per-kernel rocprofv3 averages of the update at minibatch 4096
# and 64 and the update step time (train_probe.py), alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r04ab.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_r04ab.log | tail -12
[ $rc -le 1 ] || { tail -40 gpurun_out/pytest_r04ab.log; exit $rc; }
for r in 1 2 3; do
  for b in r04ab_head base; do
    KERNELS="k_wgrad k_reduce_grads k_adam" TAG=r04ab_$r bash scripts/ab_kernel_time.sh $b || exit 1
    BS=64 MAXSTEPS=256 N=16384 KERNELS="k_wgrad k_reduce_grads k_adam" TAG=r04ab64_$r bash scripts/ab_kernel_time.sh $b || exit 1
  done
done
cd $GRAFT_REPO_ROOT
bash scripts/ab_train_quick.sh r04ab_head base || exit 1
echo all done
