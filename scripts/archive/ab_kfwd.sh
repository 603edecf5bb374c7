# Per-kernel A/B at minibatch 4096 (forward-TR, K6, k_wgrad) for the builds given, two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  BS=4096 N=65536 MAXSTEPS=16 bash scripts/ab_kstats.sh "$@" > /dev/null 2>&1 || exit 1
  for b in "$@"; do python3 -c "
import csv
d={r['Name'].split('(')[0].replace('void ','').split('::')[-1][:24]: float(r['AverageNs'])/1000 for r in csv.DictReader(open('gpurun_out/ab_$b/run_kernel_stats.csv'))}
print('round $r $b', {k: round(v,1) for k,v in d.items() if k.startswith(('k_policy_forward','k_policy_backward','k_wgrad','k_reduce','k_adam'))})"; done
done
