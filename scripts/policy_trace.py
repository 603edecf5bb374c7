"""Phase timeline of k_policy_forward from a TRACE=1 build (make -C .../csrc TRACE=1).

Runs the fused forward at B windows, reads the s_memtime stamps of waves 0 and 4 of the first
256 workgroups and prints the median cycles spent between consecutive phase boundaries.
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

NAMES = {0: "start", 1: "x+mask", 2: "a.embed", 3: "a.layer+sync", 4: "a.head", 5: "c.layers+sync", 6: "c.head",
         7: "sample", 60: "env.sync", 61: "env.loads", 62: "env.step", 63: "env.store",
         55: "C0.LN1 acc ready", 56: "C0.LN1 partials", 57: "C0.LN1 barrier", 23: "C0.LN2 acc ready",
         39: "C0.LN2 partials", 58: "C0.LN2 barrier"}
ENVFINE = {40: "g.pair reads", 41: "g.rev loop", 42: "g.accept", 43: "g.rew/done", 44: "g.pair+push_obs",
           45: "g.write_obs"}
LAYER = ["start", "c0 gemm", "c0 sync", "c0 attn+sync", "c1 gemm", "c1 sync", "c1 attn+sync", "outproj", "sync",
         "LN1+sync", "FFN1", "sync", "FFN2+sync", "store+sync", "LN2"]
for li, tag in enumerate(["A", "C0", "C1"]):
    for j, n in enumerate(LAYER):
        NAMES[8 + 16 * li + j] = f"{tag}.{n}"
    NAMES[8 + 16 * li + 13] = f"{tag}.ring gemm"
if os.environ.get("ENVFINE") == "1":  # a make TRACE=1 ENVFINE=1 build: stamps inside the env step
    NAMES.update(ENVFINE)

B = int(os.environ.get("B", "4096"))
torch.manual_seed(0)
net = TransformerActorCritic().cuda()
x = torch.randn(B, 5, 14, device="cuda")
x[: B // 4, :2] = 0
a = torch.empty(B, dtype=torch.int8, device="cuda")
lp = torch.empty(B, device="cuda")
v = torch.empty(B, device="cuda")
STEPS = os.environ.get("STEPS", "0") == "1"  # k_rollout_steps (one launch of 8 steps; last step's stamps)
fn = _lib.LIB.uavhip_steps_trace if STEPS else _lib.LIB.uavhip_policy_trace
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
ROWS = os.environ.get("ROWS", "0") == "1"  # window-row ring path (uavhip_policy_forward_rows)
ENV = os.environ.get("ENV", "0") == "1" or STEPS  # fused rollout step (uavhip_rollout_step), 16 x 32 envs
kw = {}
if ENV:  # the stamps of the last of 8 fused steps
    from uavhip import VecUAVEnv
    from uavhip.rollout import RolloutEngine
    env = VecUAVEnv(B, 16, 32, 1, 1, seed=1)
    eng = RolloutEngine(env, net, horizon=8)
    eng.start()
    tr = eng.traj
    tr.obs[0].copy_(tr.obs[8])
    if STEPS:
        net.rollout_steps(env, tr.obs[:9].contiguous(), eng.rowproj, 0, True, tr.actions[:8], tr.logp[:8],
                          tr.values[:8], tr.rewards[:8], tr.dones[:8], tr.info[:8], seed=0, offset=0,
                          offset_stride=B, offset_dev=eng.counter)
    for t in range(0 if STEPS else 8):
        net.rollout_step(env, tr.obs[t], eng.rowproj, t, t == 0, tr.actions[t], tr.logp[t], tr.values[t],
                         tr.obs[t + 1], tr.rewards[t], tr.dones[t], seed=0, offset=t * B, offset_dev=eng.counter)
elif ROWS:
    from uavhip.policy import rowproj_buffer
    rp = rowproj_buffer(B)
for i in range(0 if ENV else 5):
    if ROWS:  # timing only: the same windows replayed as a sequence
        kw = dict(rowproj=rp, step=i, fill=i == 0)
    net.fused_forward(x, action_out=a, logp=lp, value=v, **kw)
torch.cuda.synchronize()
buf = np.zeros(256 * 2 * 64, np.uint64)
assert fn(buf.ctypes.data, buf.size) == 0
if os.environ.get("WAVES") == "8":  # a TRACE_WAVES=8 build: [64 workgroups][8 waves][slots]
    t8 = buf.reshape(64, 8, 64).astype(np.int64)
    slots = sorted((k for k in NAMES if (t8[:, :, k] != 0).all()),
                   key=lambda k: np.median(t8[:, 0, k] - t8[:, 0, 0]))
    rel = t8 - t8[:, 0:1, 0:1]  # every wave against wave 0's block start
    print(f"B={B}; median cycles since block start, waves 0-7 (64 workgroups)")
    for k in slots:
        print(f"{k:3d} {NAMES[k]:18s} " + " ".join(f"{int(np.median(rel[:, w, k])):7d}" for w in range(8)))
    sys.exit(0)
t = buf.reshape(256, 2, 64).astype(np.int64)
slots = sorted((k for k in NAMES if (t[:, 0, k] != 0).all() and k not in ENVFINE), key=lambda k: np.median(t[:, 0, k] - t[:, 0, 0]))
base = t[:, :, 0:1]
rel = t - base
print(f"B={B}; median cycles since block start (wave0 / wave4) and per-phase delta (wave0)")
prev = 0
for k in slots:
    m0 = int(np.median(rel[:, 0, k]))
    m4 = int(np.median(rel[:, 1, k])) if (t[:, 1, k] != 0).all() else -1
    print(f"{k:3d} {NAMES[k]:18s} {m0:8d} {m4:8d}  +{m0 - prev:6d}")
    prev = m0
if os.environ.get("ENVFINE") == "1":  # conditional stamps: only blocks whose stamp lies in this step's env step
    print("env step detail (wave 0; median cycles since env.loads over the blocks that stamped the slot)")
    for k in sorted(ENVFINE):
        ok = (t[:, 0, k] >= t[:, 0, 61]) & (t[:, 0, k] <= t[:, 0, 62])
        if ok.any():
            print(f"{k:3d} {ENVFINE[k]:18s} {int(np.median(t[ok, 0, k] - t[ok, 0, 61])):8d}  ({int(ok.sum())} blocks)")
start = t[:, 0, 0]
end = t[:, 0, 63 if ENV else 7]
dur = (t[:, 0, 63 if ENV else 7] - t[:, 0, 0]).astype(np.float64)
q = np.percentile(dur, [0, 10, 50, 90, 99, 100])
print("per-block duration (wave 0, cycles): min %d p10 %d median %d p90 %d p99 %d max %d; max/median %.3f"
      % (*q, q[5] / q[2]))
print(f"block start spread {int(start.max() - start.min())} cycles; end spread {int(end.max() - end.min())};"
      f" kernel span {int(end.max() - start.min())} cycles")
