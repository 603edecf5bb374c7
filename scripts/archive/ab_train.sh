#!/bin/bash
# PPO training-step timing for several builds on one box, alternating (GPU box):
#   bash scripts/ab_train.sh exp_a exp_b ...   ("base" = the in-tree library)
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
  for x in "$@"; do
    lib=""; [ "$x" != base ] && lib="$PWD/scripts/$x/libuavhip.so"
    echo -n "$x: "
    UAVHIP_LIB=$lib BS=${BS:-4096,64} EPOCHS=${EPOCHS:-3} timeout -k 10 200 python scripts/train_probe.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1
    echo
  done
done
