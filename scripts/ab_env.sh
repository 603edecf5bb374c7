#!/bin/bash
# A/B of the env-only fused line (scripts/env_probe.py) between the product build and scripts/$1
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for lib in "" "$PWD/scripts/$1/libuavhip.so"; do
    echo "lib=${lib:-base}"
    UAVHIP_LIB=$lib E=4096 N=16 M=32 T=256 REPS=10 timeout -k 10 100 python scripts/env_probe.py || exit 1
  done
done
