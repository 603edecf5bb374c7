"""Phase cycles of K2r (k_env_replay) from a TRACE=1 build: walk, fold, replay, carried state,
barrier wait (the store waves work beside), per chunk (means over the traced envs), at BASELINE configs[1] (1024 x 8 x 16) and the
headline shape (4096 x 16 x 32), T = 256, every output written.
Usage (GPU box): UAVHIP_LIB=$PWD/scripts/trace_lib/libuavhip.so python scripts/env_trace_probe.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "target-allocation-ppo-transformer_amd")]
from uavhip import _lib  # noqa: E402
from uavhip.vec_env import VecUAVEnv  # noqa: E402

PH = ("walk", "fold", "replay", "carry", "sync")
fn = _lib.LIB.uavhip_env_trace
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
for (E, N, M, T) in [(1024, 8, 16, 256), (4096, 16, 32, 256)]:
    v = VecUAVEnv(E, N, M, 1, 1, seed=77, full_reset_period=200)
    v.istate[:, 4] = 1
    v.generate_scenes()
    v.reset(episode=1)
    acts = torch.randint(0, 2, (T, E), generator=torch.Generator(device="cuda").manual_seed(5), device="cuda",
                         dtype=torch.int8)
    outs = dict(obs_out=torch.empty(T, E, 5, 14, device="cuda"),
                reward_out=torch.empty(T, E, dtype=torch.float64, device="cuda"),
                done_out=torch.empty(T, E, dtype=torch.uint8, device="cuda"),
                info_out=torch.empty(T, E, 8, dtype=torch.float64, device="cuda"))
    for _ in range(3):
        v.step(acts, **outs)
        v.refresh_scenes()
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 6, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(4096, 6)[:E].astype(np.float64)
    chunks = t[:, 5]
    per = t[:, :5] / chunks[:, None]
    tot = per.sum(1)
    print(f"{E}x{N}x{M} T={T}: {chunks.mean():.1f} chunks/wave, cycles per chunk: total {tot.mean():.0f} ("
          + ", ".join(f"{p} {per[:, i].mean():.0f}" for i, p in enumerate(PH)) + f"); per step {tot.mean() * chunks.mean() / T:.0f}")
