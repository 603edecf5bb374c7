"""Minimal driver for profiling k_policy_forward alone: B windows, N launches."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "target-allocation-ppo-transformer_amd"))
import torch  # noqa: E402
from uavhip.policy import TransformerActorCritic  # noqa: E402

B = int(os.environ.get("B", "4096"))
N = int(os.environ.get("N", "20"))
torch.manual_seed(0)
net = TransformerActorCritic().cuda()
x = torch.randn(B, 5, 14, device="cuda")
x[: B // 4, :2] = 0
a = torch.empty(B, dtype=torch.int8, device="cuda")
lp = torch.empty(B, device="cuda")
v = torch.empty(B, device="cuda")
for _ in range(3):
    net.fused_forward(x, action_out=a, logp=lp, value=v)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    net.fused_forward(x, action_out=a, logp=lp, value=v)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / N
print(f"B={B} avg {dt * 1e6:.1f} us/launch  {2446208 * B / dt / 1e12:.1f} TFLOP/s")
