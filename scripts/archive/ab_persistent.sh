#!/bin/bash
# Same-box A/B of the headline rollout: one launch per iteration (uavhip_rollout_steps) against one
# fused launch per step (--per-step-launch). GPU box: bash scripts/ab_persistent.sh
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for mode in "" "--per-step-launch"; do
    timeout -k 10 300 python bench.py --no-ppo --no-env-fused --no-cpu-baseline --steps 20 --warmup 3 $mode \
      > gpurun_out/ab_p.json 2> gpurun_out/ab_p.err || { tail -20 gpurun_out/ab_p.err; exit 1; }
    python - "$mode" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_p.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1] or 'persistent':20s} {d['value'] / 1e6:7.2f} M env-steps/s  ms/iter {d['ms_per_step']:.3f}  "
      f"per-step {d['roofline']['avg_launch_ms'] * 1e3:.2f} us  frac {d['roofline']['frac']:.3f}", flush=True)
PY
  done
done
