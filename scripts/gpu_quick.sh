#!/bin/bash
# quick GPU check: the gpu tests of the given files (default: all) + rollout bench without PPO / CPU legs
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
FILES=${FILES:-tests}
timeout -k 10 500 python -u -m pytest $FILES -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_quick.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ppo $BENCH_ARGS > gpurun_out/bench_q.log 2>&1
