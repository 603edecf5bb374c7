"""Timing probe for the HIP PPO training step: FusedPPOTrainer.run over n samples, per minibatch size."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "target-allocation-ppo-transformer_amd"))
import torch  # noqa: E402
from uavhip.policy import TransformerActorCritic  # noqa: E402
from uavhip.train import FusedPPOTrainer  # noqa: E402

dev = torch.device("cuda")
n = int(os.environ.get("N", "262144"))
epochs = int(os.environ.get("EPOCHS", "1"))
torch.manual_seed(0)
g = torch.Generator(device="cpu").manual_seed(5)
states = torch.randn(n, 5, 14, generator=g).to(dev)
states[: n // 8, :3] = 0
acts = torch.randint(0, 2, (n,), generator=g).to(dev)
logp = (-0.69 + 0.05 * torch.randn(n, generator=g)).to(dev)
vals = torch.randn(n, generator=g).to(dev)
ret = vals + 0.3 * torch.randn(n, device=dev)
adv = torch.randn(n, device=dev)
for bs in [int(x) for x in os.environ.get("BS", "4096,1024,64").split(",")]:
    m = min(n, bs * int(os.environ.get("MAXSTEPS", "64")))
    net = TransformerActorCritic().to(dev)
    tr = FusedPPOTrainer(net, bs)
    tr.set_buffers(states[:m], acts[:m], logp[:m], vals[:m], ret[:m], adv[:m])
    tr.capture()
    tr.run(epochs=1, generator=torch.Generator().manual_seed(1))  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = tr.run(epochs=epochs, generator=torch.Generator().manual_seed(2))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = out[3]
    print(f"bs={bs:5d} samples={m} epochs={epochs}: {dt / steps * 1e3:.3f} ms/step, "
          f"{m * epochs / dt:,.0f} sample-epochs/s, {m / dt:,.0f} PPO samples/s (5 epochs: {m / (dt / epochs * 5):,.0f})"
          f"  losses {out[0]:.4f} {out[1]:.4f} {out[2]:.4f}", flush=True)
