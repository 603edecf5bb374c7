# Same-box A/B of the bench's PPO legs (ppo_samples_per_s, minibatch-64 ms per step, rollout ms per step) for the
# in-tree build (base) against scripts/v_prev/ (UAVHIP_LIB), three alternating rounds.
#   bash scripts/ppo_ab.sh   (inside gpurun; build v_prev first: scripts/build_variant.sh v_prev <rev>)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="--steps 2 --warmup 1 --no-env-fused --no-cpu-baseline --no-e2e --no-env-diff --no-dropin"
for r in 1 2 3; do
  for b in base v_prev; do
    if [ $b = base ]; then unset UAVHIP_LIB UAVHIP_ACCEPT_PREV_ABI; else export UAVHIP_LIB=$GRAFT_REPO_ROOT/scripts/$b/libuavhip.so UAVHIP_ACCEPT_PREV_ABI=1; fi
    timeout -k 10 300 python bench.py $A > gpurun_out/ppoab_$b$r.json 2> gpurun_out/ppoab_$b$r.err || { tail -5 gpurun_out/ppoab_$b$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ppoab_$b$r.json').read().strip().splitlines()[-1]); print('$b', $r, round(d['ppo_samples_per_s']['value']/1e6,4), round(d['ppo_samples_per_s_mb64']['ms_per_optimizer_step'],5), round(d['roofline']['avg_launch_ms']*1e3,2))"
  done
done
