"""Env-only fused step probe (bench.py env_fused_rate shape) for rocprofv3 counter passes:
E envs x N UAV x M targets, T fused steps per launch, REPS launches. ACT=0/1 forces every action
(instruction-mix experiments), default Bernoulli(0.5) as in the bench."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "target-allocation-ppo-transformer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from uavhip.vec_env import VecUAVEnv  # noqa: E402

E, N, M, T = (int(os.environ.get(k, d)) for k, d in (("E", 4096), ("N", 16), ("M", 32), ("T", 64)))
reps = int(os.environ.get("REPS", "5"))
dev = torch.device("cuda")
env = VecUAVEnv(E, N, M, 1, 1, seed=77, full_reset_period=200)
env.generate_scenes()
env.reset(episode=1)
g = torch.Generator(device=dev).manual_seed(5)
acts = torch.randint(0, 2, (T, E), generator=g, device=dev, dtype=torch.int8)
if "ACT" in os.environ:
    acts.fill_(int(os.environ["ACT"]))
obs = torch.empty(T, E, 5, 14, device=dev)
rew = torch.empty(T, E, dtype=torch.float64, device=dev)
done = torch.empty(T, E, dtype=torch.uint8, device=dev)
info = torch.empty(T, E, 8, dtype=torch.float64, device=dev)
ms = []
for i in range(reps + 2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    env.step(acts, obs_out=obs, reward_out=rew, done_out=done, info_out=info)
    e1.record()
    env.refresh_scenes()
    torch.cuda.synchronize()
    if i >= 2:
        ms.append(e0.elapsed_time(e1))
t = float(np.median(ms)) * 1e-3
print(f"E={E} N={N} M={M} T={T} ACT={os.environ.get('ACT', 'rand')}: {t * 1e3:.3f} ms/launch, "
      f"{E * T / t / 1e9:.3f} G env-steps/s", flush=True)
