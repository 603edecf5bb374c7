"""Env-only fused step probe (bench.py env_fused_rate shape) for rocprofv3 counter passes:
E envs x N UAV x M targets, T fused steps per launch, REPS launches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "target-allocation-ppo-transformer_amd"))
import torch  # noqa: E402
import bench  # noqa: E402

E, N, M, T = (int(os.environ.get(k, d)) for k, d in (("E", 4096), ("N", 16), ("M", 32), ("T", 64)))
r = bench.env_fused_rate(E, N, M, T, torch.device("cuda"), reps=int(os.environ.get("REPS", "5")))
print(r, flush=True)
