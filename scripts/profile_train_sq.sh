#!/bin/bash
# SQ counters (instruction mix, stalls, MFMA busy, LDS) of the kernels of the HIP PPO training
# step (scripts/train_probe.py, minibatch 4096, 16 steps). Usage (GPU box): TAG=x bash scripts/profile_train_sq.sh
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r01}"
OUT="$R/gpurun_out/prof_trsq_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export BS=4096 MAXSTEPS=16 N=65536
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc$i" -o run -- python3 "$R/scripts/train_probe.py" > "$OUT/pmc$i.log" 2>&1 || exit $?
done
echo done > "$OUT/DONE"
