# Round-3 final measurement call: rollout phase trace (TRACE build), the full bench line, rocprofv3
# kernel stats + FETCH / WRITE PMC passes of the bench (profile.sh) and of the minibatch-4096 training
# step (profile_train.sh), and the kernel stats of the minibatch-64 (K7) training step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r03c}
UAVHIP_LIB=$PWD/target-allocation-ppo-transformer_amd/uavhip/libuavhip_trace.so STEPS=1 timeout -k 10 120 python scripts/policy_trace.py > gpurun_out/trace_steps.log 2>&1 || { tail -5 gpurun_out/trace_steps.log; exit 1; }
echo trace ok
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
echo bench ok
TAG=$TAG bash scripts/profile.sh || exit 1
echo profile ok
cd $GRAFT_REPO_ROOT
TAG=$TAG bash scripts/profile_train.sh || exit 1
echo profile_train ok
cd /tmp && export TMPDIR=/tmp
BS=64 N=16384 MAXSTEPS=256 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_train64_$TAG -o run -- python3 $GRAFT_REPO_ROOT/scripts/train_probe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_train64_$TAG.log 2>&1 || exit 1
echo done
