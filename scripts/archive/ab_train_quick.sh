#!/bin/bash
# Same-box A/B of the PPO update step (train_probe.py, minibatch 4096 and 64) across builds:
# bash scripts/ab_train_quick.sh base <build> ...  (build = scripts/<build>/libuavhip.so)
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for b in "$@"; do
    if [ "$b" = base ]; then unset UAVHIP_LIB; else export UAVHIP_LIB=$PWD/scripts/$b/libuavhip.so; fi
    echo "round $r $b"; BS=4096,64 MAXSTEPS=64 N=262144 EPOCHS=2 timeout -k 10 200 python scripts/train_probe.py 2>&1 | grep bs= || exit 1
  done
done
