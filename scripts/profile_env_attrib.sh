#!/bin/bash
# Per-buffer attribution of the env step inside k_rollout_steps: rocprofv3
# kernel-trace stats and separate PMC passes (FETCH_SIZE; WRITE_SIZE; L2 hits / misses and the
# memory-side read requests) of scripts/rollout_run.py on the product build, the NOENV build and the
# attribution builds EXP=21..27 (env_group.hpp kAttr: each compiles out one group of the env step's
# global accesses; profiling only, wrong results). Build them on the CPU first:
#   for n in 21 22 23 24 25 26 27 32; do make -C target-allocation-ppo-transformer_amd/csrc EXP=$n \
#     BUILD=build_exp$n OUT=../uavhip/libuavhip_exp$n.so; done
# Usage (GPU box): TAG=r04 bash scripts/profile_env_attrib.sh ; then
#   python scripts/summarize_env_attrib.py gpurun_out/envattr_r04 r04
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r04}"
OUT="$R/gpurun_out/envattr_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
L="$R/target-allocation-ppo-transformer_amd/uavhip"
for b in ${BUILDS:-product noenv exp21 exp22 exp23 exp24 exp25 exp26 exp27 exp32}; do
  mkdir -p "$OUT/$b"
  if [ "$b" = product ]; then export UAVHIP_LIB="$L/libuavhip.so"; else export UAVHIP_LIB="$L/libuavhip_$b.so"; fi
  [ -f "$UAVHIP_LIB" ] || { echo "missing $UAVHIP_LIB"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$b/trace" -o run -- python3 "$R/scripts/rollout_run.py" > "$OUT/$b/trace.log" 2>&1 || exit $?
  i=0
  for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/$b/pmc_$i" -o run -- python3 "$R/scripts/rollout_run.py" > "$OUT/$b/pmc_$i.log" 2>&1 || exit $?
  done
  echo "$b done"
done
echo done > "$OUT/DONE"
