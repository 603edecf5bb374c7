#!/bin/bash
# The env step inside k_rollout_steps, priced by what it adds: rocprofv3 kernel-trace stats and
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) of scripts/rollout_run.py on the product build and on
# a build with the env step compiled out (NOENV=1, profiling only, wrong results). Build the NOENV
# library on the CPU first:
#   make -C target-allocation-ppo-transformer_amd/csrc NOENV=1 BUILD=build_noenv OUT=../uavhip/libuavhip_noenv.so
# Usage (GPU box): TAG=r03 bash scripts/profile_env_share.sh ; then
#   python scripts/summarize_env_share.py gpurun_out/envshare_r03 r03
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r03}"
OUT="$R/gpurun_out/envshare_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for b in product noenv; do
  mkdir -p "$OUT/$b"
  if [ "$b" = product ]; then export UAVHIP_LIB="$R/target-allocation-ppo-transformer_amd/uavhip/libuavhip.so";
  else export UAVHIP_LIB="$R/target-allocation-ppo-transformer_amd/uavhip/libuavhip_noenv.so"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$b/trace" -o run -- python3 "$R/scripts/rollout_run.py" > "$OUT/$b/trace.log" 2>&1 || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/$b/pmc_$c" -o run -- python3 "$R/scripts/rollout_run.py" > "$OUT/$b/pmc_$c.log" 2>&1 || exit $?
  done
done
echo done > "$OUT/DONE"
