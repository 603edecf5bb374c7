# Same-box kernel-time A/B of the PPO training step (scripts/train_probe.py under rocprofv3
# --kernel-trace --stats) for the in-tree build and the builds named in AB (scripts/<name>/libuavhip.so).
#   TAG=r05l AB="v_r4" BS=64 bash scripts/gpu_train_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-trab}
export BS=${BS:-64} MAXSTEPS=${MAXSTEPS:-64} N=${N:-65536}
cd /tmp && export TMPDIR=/tmp
for b in base $AB; do
  OUT=$GRAFT_REPO_ROOT/gpurun_out/trab_${TAG}_$b
  mkdir -p $OUT
  if [ $b = base ]; then unset UAVHIP_LIB; else export UAVHIP_LIB=$GRAFT_REPO_ROOT/scripts/$b/libuavhip.so UAVHIP_ACCEPT_PREV_ABI=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/scripts/train_probe.py > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
  echo "== $b"; grep "bs=" $OUT/probe.log
  python3 - $OUT <<'EOF'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(f"  {r['Name'][:48]:48s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.2f} us")
EOF
done
