#!/bin/bash
# rocprofv3 kernel stats + SQ instruction / stall counters of the env-only fused step
# (scripts/env_probe.py). Usage (GPU box): TAG=r01 bash scripts/profile_env.sh
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r01}"
OUT="$R/gpurun_out/prof_env_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/scripts/env_probe.py" > "$OUT/trace.log" 2>&1 || exit $?
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc$i" -o run -- python3 "$R/scripts/env_probe.py" > "$OUT/pmc$i.log" 2>&1 || exit $?
done
echo done > "$OUT/DONE"
