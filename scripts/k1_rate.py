"""K1 (k_score_pairs) pairs/s at BASELINE configs[4]'s shape (8192 envs x 64 UAVs x 128 targets) and
the headline shape, median of 7 launches (HIP events); UAVHIP_LIB selects the build (A/B runs)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = ["bench.py"]
import torch  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
out = {}
for E, N, M in ((8192, 64, 128), (4096, 16, 32)):
    r = bench.score_pairs_rate(E, N, M, dev, reps=7)
    out[f"{E}x{N}x{M}"] = {"pairs_per_s": r["value"], "ms": r["ms_per_launch"]}
print(json.dumps({"lib": os.environ.get("UAVHIP_LIB", "in-tree"), **out}))
