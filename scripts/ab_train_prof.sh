#!/bin/bash
# Per-kernel A/B of the training step: rocprofv3 kernel stats of scripts/train_probe.py with the
# product build and with scripts/$1
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
export BS=4096 MAXSTEPS=32 N=131072
for x in base "$1" base "$1"; do
  lib=""; [ "$x" != base ] && lib="$R/scripts/$x/libuavhip.so"
  UAVHIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/abp_$x$((i=i+1))" -o run -- python3 "$R/scripts/train_probe.py" > "$R/gpurun_out/abp_$x.log" 2>&1 || exit 1
done
