#!/bin/bash
# env-kernel change check: gpu env tests + rollout bench (no PPO / CPU baseline)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_policy_gae.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_env.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ppo > gpurun_out/bench_q.log 2>&1
