# Round-4 final set, training half: the update's kernel stats + FETCH / WRITE passes at minibatch 4096
# (profile_train.sh) and the kernel stats at the reference's minibatch 64.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=r04zf bash scripts/profile_train.sh || exit 1
cd /tmp && export TMPDIR=/tmp
BS=64 MAXSTEPS=256 N=16384 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $GRAFT_REPO_ROOT/gpurun_out/prof_train64_r04zf -o run -- python3 $GRAFT_REPO_ROOT/scripts/train_probe.py \
  > $GRAFT_REPO_ROOT/gpurun_out/prof_train64_r04zf.log 2>&1 || exit 1
echo all done
