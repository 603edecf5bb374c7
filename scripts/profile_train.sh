#!/bin/bash
# rocprofv3 kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes of the HIP PPO training step
# (scripts/train_probe.py, minibatch 4096, 16 steps). Usage (GPU box): TAG=r01 bash scripts/profile_train.sh
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r01}"
OUT="$R/gpurun_out/prof_train_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export BS=4096 MAXSTEPS=16 N=65536
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/scripts/train_probe.py" > "$OUT/trace.log" 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run -- python3 "$R/scripts/train_probe.py" > "$OUT/pmc_$c.log" 2>&1 || exit $?
done
echo done > "$OUT/DONE"
