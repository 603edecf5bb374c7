import sys, torch, numpy as np
sys.path.insert(0, "target-allocation-ppo-transformer_amd")
from uavhip import _lib
from uavhip.vec_env import VecUAVEnv
for E, dt, T, period in ((8192, torch.float16, 200, 200), (8192, torch.float32, 200, 200), (4096, torch.float16, 200, 200),
                         (256, torch.float16, 200, 200), (8192, torch.float16, 1, 200), (8192, torch.float16, 200, 0)):
    v = VecUAVEnv(E, 64, 128, 1, 1, full_reset_period=period, seed=13, obs_dtype=dt)
    v.istate[:, _lib.IST["EPISODE"]] = 1
    v.generate_scenes()
    torch.cuda.synchronize()
    e0 = v.errors().clone()
    v.reset(episode=1)
    e1 = v.errors().clone()
    g = torch.Generator(device="cuda").manual_seed(12)
    acts = (torch.rand(T, E, device="cuda", generator=g) < 0.4).to(torch.int8)
    v.step(acts)
    torch.cuda.synchronize()
    e2 = v.errors()
    nz = (e2 != 0).nonzero()
    print(E, dt, T, period, "after gen", int(e0.abs().max()), "after reset", int(e1.abs().max()), "after step", int(e2.abs().max()),
          "n nonzero", int((e2 != 0).sum()), "first", nz[:3].view(-1).tolist(), "istate row", v.istate[nz[0, 0]].tolist() if len(nz) else None, flush=True)
