# The update's measurement set: kernel stats + FETCH / WRITE passes at minibatch 4096
# (profile_train.sh -> profiles/${TAG}_train_{kernel_stats.csv,pmc.json}) and the kernel stats at the
# reference's minibatch 64 (-> profiles/${TAG}_train64_kernel_stats.csv), copied to gpurun_out/profiles_$TAG.
#   TAG=r05z bash scripts/gpu_train_prof.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-train}
TAG=$TAG bash scripts/profile_train.sh || exit 1
cd $GRAFT_REPO_ROOT
python scripts/summarize_profile.py gpurun_out/prof_train_$TAG ${TAG}_train > /dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
BS=64 MAXSTEPS=256 N=16384 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $GRAFT_REPO_ROOT/gpurun_out/prof_train64_$TAG -o run -- python3 $GRAFT_REPO_ROOT/scripts/train_probe.py \
  > $GRAFT_REPO_ROOT/gpurun_out/prof_train64_$TAG.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profiles_$TAG
cp profiles/${TAG}_train_* gpurun_out/profiles_$TAG/
cp $(find gpurun_out/prof_train64_$TAG -name run_kernel_stats.csv | head -1) gpurun_out/profiles_$TAG/${TAG}_train64_kernel_stats.csv
grep "bs=" gpurun_out/prof_train_$TAG/trace.log gpurun_out/prof_train64_$TAG.log
echo train profiles done
