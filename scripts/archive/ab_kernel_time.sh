#!/bin/bash
# Per-kernel average duration (rocprofv3 kernel trace) of the training probe for several builds:
#   KERNELS="k_wgrad k_reduce" bash scripts/ab_kernel_time.sh base wexp51 ...   (GPU box)
# ("base" = the in-tree library; others scripts/<name>/libuavhip.so). Extra env goes to train_probe.py.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/ab_kernel_${TAG:-x}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export BS=${BS:-4096} MAXSTEPS=${MAXSTEPS:-16} N=${N:-65536}
for x in "$@"; do
  lib=""; [ "$x" != base ] && lib="$R/scripts/$x/libuavhip.so"
  UAVHIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$x" -o run -- python3 "$R/scripts/train_probe.py" > "$OUT/$x.log" 2>&1 || exit $?
  python3 - "$OUT/$x/run_kernel_stats.csv" "$x" ${KERNELS:-k_wgrad} <<'PY'
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
