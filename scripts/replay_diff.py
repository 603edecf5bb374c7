"""Debug aid (GPU box): first differences between K2r and K2 outputs on twin envs (the setup of
tests/test_gpu_env.py::_replay_twins), per output tensor: index and both values.
Usage: python scripts/replay_diff.py [E N M period T p]"""
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "target-allocation-ppo-transformer_amd")]
from test_gpu_env import _replay_twins  # noqa: E402

E, N, M, period, T = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (1024, 8, 16, 3, 200)))
p = float(sys.argv[6]) if len(sys.argv) > 6 else 0.5
a, b = _replay_twins(E, N, M, period, T, 3, torch.float32, p, seed=E + N + M)
names = [f"{k}{i}" for i in range(3) for k in ("obs", "rew", "done", "info")] + [
    "istate", "dstate", "window", "nh_final", "nh_pure", "t_cost", "n_lock", "assigned", "p_dmg"]
for name, x, y in zip(names, a, b):
    if torch.equal(x, y):
        continue
    d = (x != y).nonzero()
    print(f"{name}: {d.shape[0]} differing elements; first {d[:6].tolist()}")
    for idx in d[:4].tolist():
        print("   ", idx, "K2r", x[tuple(idx)].item(), "K2", y[tuple(idx)].item())
