#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_policy_${TAG:-a}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
timeout -k 10 200 python3 "$R/scripts/policy_driver.py" > "$OUT/plain.log" 2>&1 || exit $?
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex k_policy --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/scripts/policy_driver.py" > "$OUT/p$i.log" 2>&1 || exit $?
done
