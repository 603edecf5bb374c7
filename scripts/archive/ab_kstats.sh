#!/bin/bash
# Per-kernel averages (rocprofv3 --kernel-trace --stats) of scripts/train_probe.py for several builds
# on one box: bash scripts/ab_kstats.sh base exp101 ...  ("base" = the in-tree library).
# BS / N / MAXSTEPS pass through to train_probe.py (default: minibatch 64, 256 steps).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export BS=${BS:-64} N=${N:-16384} MAXSTEPS=${MAXSTEPS:-256}
cd /tmp && export TMPDIR=/tmp
for b in "$@"; do
  if [ "$b" = base ]; then unset UAVHIP_LIB; else export UAVHIP_LIB=$R/scripts/$b/libuavhip.so; fi
  out=$R/gpurun_out/ab_$b
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 $R/scripts/train_probe.py > $out.log 2>&1 || { tail -5 $out.log; exit 1; }
  echo "== $b: $(grep bs= $out.log)"
  python3 - "$out/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = 0.0
for r in rows:
    if not r['Name'].startswith('uavhip'):
        continue
    print(f"   {r['Name'].split('(')[0][:48]:48s} {int(r['Calls']):6d} avg {float(r['AverageNs'])/1000:8.2f} us")
PY
done
