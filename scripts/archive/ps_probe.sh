# Position split (K7) timing: train_probe at small minibatches with K7 on / off, then a rocprofv3
# kernel-trace of minibatch 64 (K7 on).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export BS=${BS:-64,128,256} N=${N:-262144} MAXSTEPS=${MAXSTEPS:-256}
timeout -k 10 200 python scripts/train_probe.py > gpurun_out/ps_on.log 2>&1 || { tail -20 gpurun_out/ps_on.log; exit 1; }
cat gpurun_out/ps_on.log
UAVHIP_POS_SPLIT=0 timeout -k 10 200 python scripts/train_probe.py > gpurun_out/ps_off.log 2>&1 || { tail -20 gpurun_out/ps_off.log; exit 1; }
cat gpurun_out/ps_off.log
cd /tmp && export TMPDIR=/tmp
BS=64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ps64 -o run -- python3 $GRAFT_REPO_ROOT/scripts/train_probe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_ps64.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_ps64/run_kernel_stats.csv")))
for r in rows[:14]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1000:8.2f} us")
PY
