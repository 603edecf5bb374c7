#!/bin/bash
# rocprofv3 SQ instruction / stall counters of the env-only fused step (scripts/env_probe.py) for
# random, all-skip and all-assign actions. Usage (GPU box): TAG=r01 bash scripts/profile_env.sh
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r01}"
OUT="$R/gpurun_out/prof_env_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for a in rand 0 1; do
  if [ "$a" = rand ]; then unset ACT; else export ACT=$a; fi
  timeout -k 10 300 python3 "$R/scripts/env_probe.py" >> "$OUT/rate.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM --output-format csv -d "$OUT/pmc_$a" -o run -- python3 "$R/scripts/env_probe.py" > "$OUT/pmc_$a.log" 2>&1 || exit $?
done
echo done > "$OUT/DONE"
