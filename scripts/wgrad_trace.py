"""Phase stamps of k_wgrad (TRACE=1 build): per workgroup, the first-slab wait, the k-loop and the
epilogue of each stream-K run, from one training step at BS samples."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "target-allocation-ppo-transformer_amd"))
import torch  # noqa: E402
from uavhip import _lib  # noqa: E402
from uavhip.policy import TransformerActorCritic  # noqa: E402
from uavhip.train import FusedPPOTrainer  # noqa: E402

bs = int(os.environ.get("BS", "4096"))
n = bs * 4
dev = torch.device("cuda")
g = torch.Generator().manual_seed(5)
states = torch.randn(n, 5, 14, generator=g).to(dev)
acts = torch.randint(0, 2, (n,), generator=g).to(dev)
logp = (-0.69 + 0.05 * torch.randn(n, generator=g)).to(dev)
vals = torch.randn(n, generator=g).to(dev)
tr = FusedPPOTrainer(TransformerActorCritic().to(dev), bs)
tr.set_buffers(states, acts, logp, vals, vals + 0.1, torch.randn(n, generator=g).to(dev))
tr.run(epochs=1, generator=torch.Generator().manual_seed(1), use_graph=False)
torch.cuda.synchronize()
fn = _lib.LIB.uavhip_wgrad_trace
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(256 * 16, np.uint64)
assert fn(buf.ctypes.data, buf.size) == 0
t = buf.reshape(256, 16).astype(np.int64)
t0 = t[:, 0:1]
rel = np.where(t > 0, t - t0, -1)
print("per-workgroup cycles since start (median / max over workgroups with that run)")
for r in range(3):
    cols = [1 + 4 * r, 2 + 4 * r, 3 + 4 * r]
    have = (t[:, cols[0]] > 0)
    if not have.any():
        continue
    first = rel[have, cols[0]] - (rel[have, cols[0] - 1] if r > 0 else 0)
    loop = rel[have, cols[1]] - rel[have, cols[0]]
    epi = rel[have, cols[2]] - rel[have, cols[1]]
    print(f"run {r}: workgroups {have.sum():3d}  first-slab wait {int(np.median(first)):7d}  "
          f"k-loop {int(np.median(loop)):7d}  epilogue {int(np.median(epi)):6d}")
last = np.max(np.where(t[:, 1:] > 0, t[:, 1:], 0), axis=1) - t[:, 0]
print(f"workgroup span median {int(np.median(last))} max {int(last.max())}; start spread {int(t0.max() - t0.min())}")
