#!/bin/bash
# A/B timing of an experimental build (scripts/$1/libuavhip.so) against the product build:
# rollout bench line (no PPO / CPU / env-only legs) + training-step probe, alternating A B A B.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
EXP=$1
for r in 1 2; do
  for lib in "" "$PWD/scripts/$EXP/libuavhip.so"; do
    tag=${lib:+exp}; tag=${tag:-base}
    UAVHIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-ppo --no-env-fused --steps 20 > gpurun_out/ab_bench_$tag$r.log 2>&1 || exit 1
    UAVHIP_LIB=$lib BS=4096 EPOCHS=2 timeout -k 10 200 python scripts/train_probe.py > gpurun_out/ab_train_$tag$r.log 2>&1 || exit 1
  done
done
for f in gpurun_out/ab_bench_*.log; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e6,2), round(d['roofline']['avg_launch_ms']*1e3,2))"; done
grep -h "bs=" gpurun_out/ab_train_*.log
