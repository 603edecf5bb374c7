"""Env-only multi-step launch rates (GPU box): K2r (omega = 0 replay) against the step-by-step
kernels (K2 one env per wave, K2g two per wave), with and without the observation / info outputs.
Usage: python scripts/env_rate_probe.py"""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "target-allocation-ppo-transformer_amd")]
from uavhip import _lib  # noqa: E402
from uavhip.vec_env import VecUAVEnv  # noqa: E402


def rate(E, N, M, T, flags, outs=("obs", "rew", "done", "info"), reps=5):
    v = VecUAVEnv(E, N, M, 1, 1, seed=77, full_reset_period=200)
    v.desc.flags |= flags
    v.istate[:, 4] = 1
    v.generate_scenes()
    v.reset(episode=1)
    g = torch.Generator(device="cuda").manual_seed(5)
    acts = torch.randint(0, 2, (T, E), generator=g, device="cuda", dtype=torch.int8)
    kw = dict(obs_out=torch.empty(T, E, 5, 14, device="cuda"), reward_out=torch.empty(T, E, dtype=torch.float64, device="cuda"),
              done_out=torch.empty(T, E, dtype=torch.uint8, device="cuda"),
              info_out=torch.empty(T, E, 8, dtype=torch.float64, device="cuda"))
    from uavhip._lib import LIB, check, ptr, stream_handle
    args = [kw["obs_out"] if "obs" in outs else None, kw["reward_out"] if "rew" in outs else None,
            kw["done_out"] if "done" in outs else None, kw["info_out"] if "info" in outs else None]
    def launch():
        check(LIB.uavhip_env_step(v.desc, ptr(acts), T, 1, *[ptr(a) for a in args], stream_handle()), "step")
    for _ in range(2):
        launch(); v.refresh_scenes()
    ts = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(reps):
        e0.record(); launch(); e1.record(); v.refresh_scenes(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    ms = ts[len(ts) // 2]
    return E * T / (ms * 1e-3), ms


QUICK = os.environ.get("PROBE_QUICK") == "1"  # one launch shape, full outputs (counter passes)
for (E, N, M, T) in [(1024, 8, 16, 256)] + ([] if QUICK else [(4096, 8, 16, 256), (4096, 16, 32, 256)]):
    for name, flags in (("K2r", 1), ("K2g", 4), ("K2", 5)):  # ONE_PER_WAVE keeps K2g out of the K2r leg
        for outs in (("obs", "rew", "done", "info"),) + (() if QUICK else (("rew", "done", "info"), ("rew", "done"), ())):
            r, ms = rate(E, N, M, T, flags, outs)
            print(f"{E}x{N}x{M} T={T} {name:4s} outs={','.join(outs) or '-':18s} {r / 1e9:6.3f} G env-steps/s  {ms:.4f} ms", flush=True)
