"""The env step's share of a k_rollout_steps step, from the s_memtime phase stamps of the TRACE
build (libuavhip_trace.so: make -C target-allocation-ppo-transformer_amd/csrc TRACE=1
BUILD=build_trace OUT=../uavhip/libuavhip_trace.so; __graft_entry__.build() makes it).

bench.py runs this as a child process (its own GPU context; the product library is never replaced)
and prices the env step as share x the per-step time it measured with HIP events on the product
build. Share = median over the first 256 workgroups (wave 0) of
    (env.store - sample) / (env.store - start)
of the LAST step of a 64-step launch at the bench's shape: the cycles from the end of sampling
(the barrier the env step needs, the scalar broadcasts, uav_env.py:295-435 on two envs per wave, the
state stores) over the whole step. Both stamps come from the same wave in the same launch, so the
ratio does not depend on the clock (which drops under dense MFMA issue). The env state's loads are
issued before the critic head and hide under it; they are not in the share.

Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "target-allocation-ppo-transformer_amd")
os.environ.setdefault("UAVHIP_LIB", os.path.join(PKG, "uavhip", "libuavhip_trace.so"))
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402
import torch  # noqa: E402

START, SAMPLE, ENV_SYNC, ENV_LOADS, ENV_STEP, ENV_STORE = 0, 7, 60, 61, 62, 63


def main():
    E = int(os.environ.get("E", "4096"))
    N, M, T = int(os.environ.get("N", "16")), int(os.environ.get("M", "32")), int(os.environ.get("T", "64"))
    from uavhip import _lib
    from uavhip.policy import TransformerActorCritic
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv
    if not hasattr(_lib.LIB, "uavhip_steps_trace"):
        raise SystemExit(f"{_lib.LIB_PATH} is not a TRACE build")
    fn = _lib.LIB.uavhip_steps_trace
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    torch.manual_seed(0)
    net = TransformerActorCritic().cuda()
    env = VecUAVEnv(E, N, M, 1, 1, seed=1, full_reset_period=200)
    eng = RolloutEngine(env, net, horizon=T, persistent=True)
    eng.start()
    for _ in range(3):  # the bench's steady state: the last iteration's last step is read
        eng.collect(eager=True)
    torch.cuda.synchronize()
    buf = np.zeros(256 * 2 * 64, np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(256, 2, 64).astype(np.int64)[:, 0]
    ok = (t[:, [START, SAMPLE, ENV_SYNC, ENV_STORE]] != 0).all(1)
    t = t[ok]
    step = t[:, ENV_STORE] - t[:, START]
    env_c = t[:, ENV_STORE] - t[:, SAMPLE]
    share = env_c / step
    out = {"blocks": int(ok.sum()), "step_cycles": float(np.median(step)), "env_cycles": float(np.median(env_c)),
           "share": float(np.median(share)), "share_p10": float(np.percentile(share, 10)),
           "share_p90": float(np.percentile(share, 90)),
           "phases": {k: float(np.median(t[:, b] - t[:, a])) for k, a, b in
                      (("sync", SAMPLE, ENV_SYNC), ("loads", ENV_SYNC, ENV_LOADS), ("step", ENV_LOADS, ENV_STEP),
                       ("store", ENV_STEP, ENV_STORE))},
           "shape": [E, N, M, T], "lib": os.path.basename(_lib.LIB_PATH)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
