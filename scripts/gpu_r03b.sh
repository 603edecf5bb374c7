# Round-3 measurement call: rollout phase trace (TRACE build), full bench line, rocprofv3 kernel stats
# + FETCH/WRITE PMC passes of the bench (profile.sh) and of the training step (profile_train.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
UAVHIP_LIB=$PWD/target-allocation-ppo-transformer_amd/uavhip/libuavhip_trace.so STEPS=1 timeout -k 10 120 python scripts/policy_trace.py > gpurun_out/trace_steps.log 2>&1 || { tail -5 gpurun_out/trace_steps.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
TAG=${TAG:-r03b} bash scripts/profile.sh || exit 1
cd $GRAFT_REPO_ROOT
if [ -n "${TRAIN}" ]; then TAG=${TAG:-r03b} bash scripts/profile_train.sh || exit 1; fi
echo done
