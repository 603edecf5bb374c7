# Round-4 call b: the new precision / repack tests, the env-step attribution builds (profile_env_attrib.sh)
# and the phase timelines of the training backward / forward and the rollout step (TRACE build).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_policy_gae.py -m gpu -v -s --timeout 200 --timeout-method thread -k "per_element or prescale or large_activations or overflow or repack_on_device or pack or direct_mode or replays_reference or position_split or trunk_split or deterministic" > gpurun_out/pytest_r04b.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_r04b.log | tail -2; [ $rc -le 1 ] || exit $rc
export TL=$PWD/target-allocation-ppo-transformer_amd/uavhip/libuavhip_trace.so
UAVHIP_LIB=$TL timeout -k 10 120 python scripts/train_trace.py > gpurun_out/trace_train_r04b.log 2>&1 || { tail -5 gpurun_out/trace_train_r04b.log; exit 1; }
UAVHIP_LIB=$TL STEPS=1 timeout -k 10 120 python scripts/policy_trace.py > gpurun_out/trace_steps_r04b.log 2>&1 || { tail -5 gpurun_out/trace_steps_r04b.log; exit 1; }
echo traces ok
for m in 0 1 0 1; do UAVHIP_WGRAD_DIRECT=$m BS=64 N=16384 MAXSTEPS=256 EPOCHS=3 timeout -k 10 120 python scripts/train_probe.py >> gpurun_out/probe64_direct$m.log 2>&1 || exit 1; done
tail -2 gpurun_out/probe64_direct0.log gpurun_out/probe64_direct1.log
TAG=r04b bash scripts/profile_env_attrib.sh || exit 1
echo all done
