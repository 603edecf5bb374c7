# Round-4 call v (re-entry check of the restored tree): -m gpu, smoke, the bench line, and the
# training step's kernel stats + FETCH / WRITE passes at minibatch 4096 (the update's HBM roofline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=r04v SKIP_PROFILES=1 bash scripts/gpu_r04.sh || exit 1
cd $GRAFT_REPO_ROOT
TAG=r04v bash scripts/profile_train.sh || exit 1
echo all done
