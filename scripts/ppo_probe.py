"""Timing probe for the PPO update: eager ppo_epochs vs GraphPPOUpdater, one epoch over n samples."""
import copy
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "target-allocation-ppo-transformer_amd"))
import torch  # noqa: E402
from uavhip.policy import TransformerActorCritic  # noqa: E402
from uavhip.ppo import GraphPPOUpdater, make_optimizer, ppo_epochs  # noqa: E402

dev = torch.device("cuda")
n = int(os.environ.get("N", "65536"))
torch.manual_seed(0)
base = TransformerActorCritic().to(dev)
g = torch.Generator(device="cpu").manual_seed(5)
states = torch.randn(n, 5, 14, device=dev)
states[: n // 8, :3] = 0
acts = torch.randint(0, 2, (n,), device=dev)
logp = -torch.rand(n, device=dev)
vals = torch.randn(n, device=dev)
ret = torch.randn(n, device=dev)
adv = torch.randn(n, device=dev)
for bs in [int(x) for x in os.environ.get("BS", "4096,1024,64").split(",")]:
    nb = min(n // bs, int(os.environ.get("MAXSTEPS", "64")))
    m = nb * bs
    pe = copy.deepcopy(base)
    oe = make_optimizer(pe)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ppo_epochs(pe, oe, states[:m], acts[:m], logp[:m], vals[:m], ret[:m], adv[:m], epochs=1, batch_size=bs,
               generator=torch.Generator().manual_seed(7))
    torch.cuda.synchronize()
    te = (time.perf_counter() - t0) / nb
    pg = copy.deepcopy(base)
    og = make_optimizer(pg, capturable=True)
    up = GraphPPOUpdater(pg, og, states[:m], acts[:m], logp[:m], vals[:m], ret[:m], adv[:m], bs)
    up.capture()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    up.run(epochs=1, generator=torch.Generator().manual_seed(7))
    torch.cuda.synchronize()
    tg = (time.perf_counter() - t0) / nb
    dmax = max(float((a - b).abs().max()) for a, b in zip(pe.parameters(), pg.parameters()))
    print(f"bs={bs:5d} steps={nb}: eager {te * 1e3:.3f} ms/step ({bs / te:,.0f} sample-epochs/s)  "
          f"graph {tg * 1e3:.3f} ms/step ({bs / tg:,.0f} sample-epochs/s)  max|dparam| {dmax:.2e}", flush=True)
