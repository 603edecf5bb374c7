#!/bin/bash
# env-only fused line for several builds: bash scripts/ab_env_multi.sh exp_a exp_b ...
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for x in base "$@"; do
    lib=""; [ "$x" != base ] && lib="$PWD/scripts/$x/libuavhip.so"
    echo -n "$x: "
    UAVHIP_LIB=$lib E=4096 N=16 M=32 T=256 REPS=10 timeout -k 10 100 python scripts/env_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
