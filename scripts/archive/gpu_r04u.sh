# Round-4 call u: the training forward's trunk-order mix (UAVHIP_FWD_MIX) re-measured on the spill-free
# build, with every kernel of the minibatch-4096 step, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 3; do for m in 0 1; do echo -n "fwd mix=$m: "; UAVHIP_FWD_MIX=$m KERNELS="k_policy_forward<true k_policy_backward k_wgrad k_reduce_grads k_adam" TAG=r04u_${m}_$r bash scripts/ab_kernel_time.sh base || exit 1; done; done
echo all done
