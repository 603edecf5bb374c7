#!/bin/bash
# Per-kernel average duration (rocprofv3 kernel trace) of a bare rollout (scripts/rollout_run.py: 8
# iterations at the bench's shape) for several builds, same box:
#   KERNELS="k_policy_rows_fill k_rollout_steps" bash scripts/ab_rollout_kernels.sh base <build> ...
# ("base" = the in-tree library; others scripts/<name>/libuavhip.so).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/ab_rollout_${TAG:-x}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for x in "$@"; do
  lib=""; [ "$x" != base ] && lib="$R/scripts/$x/libuavhip.so"
  UAVHIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$x" -o run -- python3 "$R/scripts/rollout_run.py" > "$OUT/$x.log" 2>&1 || exit $?
  python3 - "$OUT/$x/run_kernel_stats.csv" "$x" ${KERNELS:-k_rollout_steps} <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for k in sys.argv[3:]:
    for r in rows:
        if k in r["Name"]:
            out.append(f"{k} {float(r['AverageNs']) / 1e3:.2f} us x{r['Calls']}")
print(sys.argv[2] + ": " + "; ".join(out), flush=True)
PY
done
