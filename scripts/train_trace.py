"""Phase timeline of k_policy_backward from a TRACE=1 build (make -C .../csrc -B TRACE=1).

Runs a few PPO minibatch steps at BS samples, reads the s_memtime stamps of waves 0 and 4 of the
first 256 workgroups of the last launch and prints the median cycles between phase boundaries.
"""
import ctypes
import os
import sys

import numpy as np

# one trunk order in every workgroup, so "cycles since block start" medians line up phase by phase
# (TrainIO::mix / BwdIO::mix run half the workgroups in the other order)
os.environ.setdefault("UAVHIP_FWD_MIX", "0")
os.environ.setdefault("UAVHIP_BWD_MIX", "0")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "target-allocation-ppo-transformer_amd"))
import torch  # noqa: E402
from uavhip import _lib  # noqa: E402
from uavhip.policy import TransformerActorCritic  # noqa: E402
from uavhip.train import FusedPPOTrainer  # noqa: E402

NAMES = {0: "start", 1: "heads bwd", 2: "c.head.0", 52: "c.embed", 53: "a.head.0", 54: "a.embed",
         55: "c.emb loads", 56: "c.emb acc", 57: "a.emb loads", 58: "a.emb acc",
         59: "hb.loads+sums", 60: "hb.per-sample+sync", 61: "hb.dz+sync"}
LAYER = ["start", "LN2", "sync", "du gemm", "sync", "W1 gemm", "sync", "LN1", "sync", "Wo gemm", "sync",
         "attn0+sync", "Win0+sync", "attn1+sync", "Win1", "res+sync"]
for base, tag in ((4, "C1"), (20, "C0"), (36, "A")):
    for j, n in enumerate(LAYER):
        NAMES[base + j] = f"{tag}.{n}"

bs = int(os.environ.get("BS", "4096"))
n = bs * 4
dev = torch.device("cuda")
g = torch.Generator().manual_seed(5)
states = torch.randn(n, 5, 14, generator=g).to(dev)
states[: n // 8, :3] = 0
acts = torch.randint(0, 2, (n,), generator=g).to(dev)
logp = (-0.69 + 0.05 * torch.randn(n, generator=g)).to(dev)
vals = torch.randn(n, generator=g).to(dev)
ret = vals + 0.3 * torch.randn(n, generator=g).to(dev)
adv = torch.randn(n, generator=g).to(dev)
torch.manual_seed(0)
tr = FusedPPOTrainer(TransformerActorCritic().to(dev), bs)
tr.set_buffers(states, acts, logp, vals, ret, adv)
tr.run(epochs=1, generator=torch.Generator().manual_seed(1), use_graph=False)
torch.cuda.synchronize()
fn = _lib.LIB.uavhip_policy_btrace
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(256 * 2 * 64, np.uint64)
assert fn(buf.ctypes.data, buf.size) == 0
t = buf.reshape(256, 2, 64).astype(np.int64)
t = t[:min(256, bs // 16)]
slots = sorted((k for k in NAMES if (t[:, 0, k] != 0).all()), key=lambda k: np.median(t[:, 0, k] - t[:, 0, 0]))
rel = t - t[:, :, 0:1]
print(f"BS={bs}; median cycles since block start (wave0 / wave4) and per-phase delta (wave0)")
prev = 0
for k in slots:
    m0 = int(np.median(rel[:, 0, k]))
    m4 = int(np.median(rel[:, 1, k])) if (t[:, 1, k] != 0).all() else -1
    print(f"{k:3d} {NAMES[k]:16s} {m0:8d} {m4:8d}  +{m0 - prev:6d}")
    prev = m0

# the training forward (k_policy_forward<TR>) of the same steps: stamps of policy_trace.py's slots
fwd = _lib.LIB.uavhip_policy_trace
fwd.restype = ctypes.c_int
fwd.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(256 * 2 * 64, np.uint64)
assert fwd(buf.ctypes.data, buf.size) == 0
t = buf.reshape(256, 2, 64).astype(np.int64)[:min(256, bs // 16)]
FN = {0: "start", 1: "x+mask", 2: "a.embed", 3: "a.layer+sync", 4: "a.head", 5: "c.layers+sync", 6: "c.head"}
FL = ["start", "c0 gemm", "c0 sync", "c0 attn+sync", "c1 gemm", "c1 sync", "c1 attn+sync", "outproj", "sync",
      "LN1+sync", "FFN1", "sync", "FFN2+sync", "store+sync", "LN2"]
for li, tag in enumerate(["A", "C0", "C1"]):
    for j, nm in enumerate(FL):
        FN[8 + 16 * li + j] = f"{tag}.{nm}"
slots = sorted(k for k in FN if (t[:, 0, k] != 0).all())
rel = t - t[:, :, 0:1]
print("training forward:")
prev = 0
for k in slots:
    m0 = int(np.median(rel[:, 0, k]))
    print(f"{k:3d} {FN[k]:16s} {m0:8d}  +{m0 - prev:6d}")
    prev = m0
