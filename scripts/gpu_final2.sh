# Second half of a round's final measurement set (after scripts/gpu_measure.sh in the previous call):
# the env-kernel counters (profile_env_counters.sh -> profiles/${TAG}_env_counters.json) and the update
# profiles (gpu_train_prof.sh -> profiles/${TAG}_train_*), copied to gpurun_out/profiles_$TAG/.
#   TAG=r06z bash scripts/gpu_final2.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r06z}
TAG=$TAG timeout -k 10 600 bash scripts/profile_env_counters.sh || exit 1
cd $GRAFT_REPO_ROOT
python scripts/summarize_env_counters.py gpurun_out/prof_env_$TAG profiles/${TAG}_env_counters.json > /dev/null || exit 1
echo env counters ok
TAG=$TAG timeout -k 10 900 bash scripts/gpu_train_prof.sh 2>&1 | tail -3 || exit 1
mkdir -p gpurun_out/profiles_$TAG
cp profiles/${TAG}_* gpurun_out/profiles_$TAG/
echo final2 ok
