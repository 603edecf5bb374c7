# Round-3 profiles: K7 minibatch-64 timing + kernel trace (ps_probe.sh), the minibatch-4096 training
# step (profile_train.sh) and the rollout bench (profile.sh), each step under its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/ps_probe.sh > gpurun_out/ps_probe.out 2>&1 || { tail -20 gpurun_out/ps_probe.out; exit 1; }
cat gpurun_out/ps_probe.out
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03} bash scripts/profile_train.sh || exit 1
cd $GRAFT_REPO_ROOT
if [ -n "${ROLLOUT}" ]; then TAG=${TAG:-r03} bash scripts/profile.sh || exit 1; fi
echo ok
