"""A/B timing of the headline rollout across library builds on one GPU box (box-to-box spread is
2-4 %, so builds are compared on the same box, alternating).

Usage (GPU box): python scripts/ab_rollout.py [build ...]   (build = scripts/<build>/libuavhip.so;
"base" = the in-tree library). Each run is a child `bench.py --no-ppo --no-env-fused
--no-cpu-baseline` process; prints the fused-step HIP-event average and env-steps/s per run.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
builds = sys.argv[1:] or ["base"]
rounds = int(os.environ.get("ROUNDS", "2"))
extra = os.environ.get("EXTRA", "").split()
res = {b: [] for b in builds}
for r in range(rounds):
    for b in builds:
        env = dict(os.environ)
        env.pop("UAVHIP_LIB", None)
        if b != "base":
            env["UAVHIP_LIB"] = os.path.join(ROOT, "scripts", b, "libuavhip.so")
            env["UAVHIP_ACCEPT_PREV_ABI"] = "1"
        out = subprocess.run([sys.executable, "bench.py", "--no-ppo", "--no-env-fused", "--no-cpu-baseline", "--no-env-diff",
                              "--no-dropin", "--no-e2e",
                              "--steps", "20", "--warmup", "3", *extra], cwd=ROOT, env=env, capture_output=True,
                             text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:])
            sys.exit(out.returncode)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        us = d["roofline"]["avg_launch_ms"] * 1e3
        res[b].append(us)
        print(f"round {r} {b:10s} fused step {us:7.2f} us  frac {d['roofline']['frac']:.3f}  "
              f"{d['value'] / 1e6:7.2f} M env-steps/s", flush=True)
for b in builds:
    print(f"{b:10s} min {min(res[b]):7.2f} us  mean {sum(res[b]) / len(res[b]):7.2f} us")
