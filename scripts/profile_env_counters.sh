#!/bin/bash
# rocprofv3 passes over the env kernels of the bench line (scripts/env_kernels_probe.py): kernel
# trace, FETCH_SIZE, WRITE_SIZE, and the VALU side (instruction counts, fp64 op mix, busy cycles).
# Usage (GPU box): TAG=r02 bash scripts/profile_env_counters.sh; then
# python scripts/summarize_env_counters.py gpurun_out/prof_env_$TAG profiles/${TAG}_env_counters.json
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r02}"
OUT="$R/gpurun_out/prof_env_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P="$R/scripts/env_kernels_probe.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$P" > "$OUT/trace.log" 2>&1 || exit $?
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES" \
         "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$i" -o run -- python3 "$P" > "$OUT/pmc_$i.log" 2>&1 || exit $?
done
echo done > "$OUT/DONE"
