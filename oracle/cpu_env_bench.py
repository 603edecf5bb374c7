"""CPU baseline of UAVEnv.step on all host cores (bench.py's cpu_baseline leg; test infrastructure).

The reference's env.step (envs/uav_env.py:295-435, recompute-from-scratch algorithm) as the C
oracle's batched loop (uo_envs_run), random Bernoulli(0.5) actions, state-only resets, one process
per core, each with its own envs and host-generated scenes (uavhip/scene.py: the reference's
_generate_scene distribution). Run as a child process that never touches the GPU:
    python -m oracle.cpu_env_bench --procs 16 --seconds 10 --uavs 16 --targets 32
prints one JSON object {"value": env-steps/s, "cores": procs, ...}.
"""
import argparse
import importlib.util
import json
import multiprocessing as mp
import os
import random
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
UAVHIP = os.path.join(ROOT, "target-allocation-ppo-transformer_amd", "uavhip")


def _load(name):
    # the pure-numpy host modules only (the uavhip package itself loads the HIP library)
    spec = importlib.util.spec_from_file_location(f"_cpu_{name}", os.path.join(UAVHIP, f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _worker(args):
    rank, seconds, N, M, n_env = args
    import oracle
    config, scene = _load("config"), _load("scene")
    c = config.Config()
    c.NUM_UAVS, c.NUM_TARGETS = N, M
    np.random.seed(rank)
    random.seed(rank)
    prm = config.params_vector(c)
    envs = [oracle.OracleEnv(scene.generate_scene(c), prm) for _ in range(n_env)]
    for e in envs:
        e.reset()
    rng = np.random.default_rng(100 + rank)
    chunk = 64
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        acts = (rng.random((chunk, n_env)) < 0.5).astype(np.int8)
        oracle.run_envs(envs, acts)
        steps += chunk * n_env
    return steps, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--uavs", type=int, default=16)
    ap.add_argument("--targets", type=int, default=32)
    ap.add_argument("--envs-per-proc", type=int, default=8)
    a = ap.parse_args()
    with mp.get_context("fork").Pool(a.procs) as pool:
        res = pool.map(_worker, [(r, a.seconds, a.uavs, a.targets, a.envs_per_proc) for r in range(a.procs)])
    steps = sum(s for s, _ in res)
    wall = max(t for _, t in res)
    print(json.dumps({"value": steps / wall, "unit": "env-steps/s", "cores": a.procs, "kind": "port",
                      "sample": f"C oracle UAVEnv.step (reference recompute-from-scratch algorithm), {a.procs} "
                                f"processes x {a.envs_per_proc} envs of {a.uavs}x{a.targets}, random actions, "
                                f"{steps} env-steps in {wall:.1f} s"}))


if __name__ == "__main__":
    main()
