"""The env kernels of the bench line's env legs, a few launches each, for rocprofv3 counter passes
(scripts/profile_env_counters.sh): K1 score_pairs over 8192 fresh 64 x 128 scenes (BASELINE
configs[4]), the env-only multi-step launch at configs[1] (1024 x 8 x 16, T = 256: K2r), at the
headline shape (4096 x 16 x 32, T = 256: K2r, 32-step chunks) and at configs[4]'s shard (8192 x 64 x 128, fp16
obs, T = 64: K2). Same seeds and shapes as bench.py's env_fused_rate / score_pairs_rate."""
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "target-allocation-ppo-transformer_amd")]
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
print(bench.score_pairs_rate(8192, 64, 128, dev, reps=3))
print(bench.env_fused_rate(1024, 8, 16, 256, dev, reps=3))
print(bench.env_fused_rate(4096, 16, 32, 256, dev, reps=3))
print(bench.env_fused_rate(8192, 64, 128, 64, dev, reps=3, obs_dtype=torch.float16))
