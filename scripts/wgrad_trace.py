"""Phase stamps of k_wgrad from a TRACE=1 build (UAVHIP_LIB=.../libuavhip_trace.so): per workgroup,
s_memtime at its start, after its first slab landed, after the k-loop and after the epilogue
(wgrad.hpp WTR slots 0-3 of the first run). Runs a few eager PPO steps at BS samples and prints the
medians and maxima of each phase over the launch's workgroups, and the spread of their start stamps.
"""
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

bs = int(os.environ.get("BS", "64"))
n = 4 * bs
torch.manual_seed(0)
g = torch.Generator().manual_seed(1)
bufs = [torch.randn(n, 5, 14, generator=g), torch.randint(0, 2, (n,), generator=g),
        -0.69 + 0.05 * torch.randn(n, generator=g), torch.randn(n, generator=g),
        torch.randn(n, generator=g), torch.randn(n, generator=g)]
bufs = [t.cuda() for t in bufs]
tr = FusedPPOTrainer(TransformerActorCritic().cuda(), bs)
tr.set_buffers(*bufs)
idx = torch.arange(bs, dtype=torch.int32, device="cuda")
for _ in range(4):
    tr.gradients(idx)
torch.cuda.synchronize()
grid = 256
out = (ctypes.c_ulonglong * (grid * 16))()
fn = _lib.LIB.uavhip_wgrad_trace
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert fn(ctypes.addressof(out), grid * 16) == 0
st = np.array(out, dtype=np.uint64).reshape(grid, 16).astype(np.int64)
live = st[:, 0] > 0
st = st[live]
t0 = st[:, 0].min()
print(f"BS={bs}: {int(live.sum())} workgroups stamped; start spread {int(st[:, 0].max() - t0)} cycles")
for name, a, b in (("first slab landed", 0, 1), ("k-loop", 1, 2), ("epilogue", 2, 3)):
    d = st[:, b] - st[:, a]
    print(f"  {name:18s} median {int(np.median(d)):7d}  max {int(d.max()):7d} cycles")
end = st[:, 3] - t0
print(f"  last epilogue done {int(end.max())} cycles after the first start")
