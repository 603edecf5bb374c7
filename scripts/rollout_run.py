"""A bare rollout for profiling: RolloutEngine at the bench's shape (one k_rollout_steps launch of T
steps per iteration, + bootstrap forward + GAE + scene refresh), nothing else: WARM (10) graph replays,
then ITERS eager iterations each after two more replays (the bench's operating point; WARM=0: cold
eager iterations only).
UAVHIP_LIB selects the library build (product / TRACE / NOENV). Prints one JSON line: host wall time
per iteration and the median over the iterations of the k_rollout_steps launch per step (HIP events
on the launch stream, bench.py's measure). bench.py runs this as a child process on the product and
the NOENV builds to price the env step by its compiled-out differential."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "target-allocation-ppo-transformer_amd"))
import torch  # noqa: E402


def main():
    E, N, M, T = (int(os.environ.get(k, d)) for k, d in (("E", 4096), ("N", 16), ("M", 32), ("T", 64)))
    iters = int(os.environ.get("ITERS", "8"))
    from uavhip import _lib
    from uavhip.policy import TransformerActorCritic
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv
    torch.manual_seed(0)
    net = TransformerActorCritic().cuda()
    env = VecUAVEnv(E, N, M, 1, 1, seed=1, full_reset_period=200)
    eng = RolloutEngine(env, net, horizon=T, persistent=True)
    eng.start()
    eng.enable_events()
    # the headline's operating point (bench.py): the iteration replayed from a hipGraph, warm, and
    # timed on an eager iteration (HIP events) that follows graph replays
    warm_replays = int(os.environ.get("WARM", "10"))
    if warm_replays > 0:
        eng.capture()
        for _ in range(warm_replays):
            eng.collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = []
    for _ in range(iters):
        if warm_replays > 0:
            for _ in range(2):
                eng.collect()
        eng.collect(eager=True)
        torch.cuda.synchronize()
        steps.append(eng.event_ms()[0][0])
    dt = time.perf_counter() - t0
    warm = steps[1:] if len(steps) > 1 and warm_replays == 0 else steps  # cold start: drop the first
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "iters": iters, "ms_per_iter": dt / iters * 1e3,
                      "step_ms": sorted(warm)[len(warm) // 2], "step_ms_all": steps,
                      "shape": [E, N, M, T]}), flush=True)


if __name__ == "__main__":
    main()
