#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of a short bench run.
# Usage (GPU box): TAG=r01 bash scripts/profile.sh
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r01}"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps ${STEPS:-10} --warmup ${WARMUP:-2} --no-cpu-baseline --no-ppo --no-dropin --no-env-diff ${EXTRA}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/trace.log" 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_$c.log" 2>&1 || exit $?
done
echo done > "$OUT/DONE"
