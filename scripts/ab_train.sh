#!/bin/bash
# A/B of the training step (scripts/train_probe.py, minibatch 4096) between the product build and scripts/$1
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2 3 4 5; do
  for lib in "" "$PWD/scripts/$1/libuavhip.so"; do
    echo -n "${lib:+exp}${lib:-base} "
    UAVHIP_LIB=$lib BS=4096 EPOCHS=2 timeout -k 10 200 python scripts/train_probe.py 2>&1 | grep "bs=" || exit 1
  done
done
