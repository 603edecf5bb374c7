"""ORACLE (test infrastructure / bench baseline only): the CPU port of the reference's own training
loop (main_train.py:79-146) at E = 1, timed on the host -- the baseline bench.py's `dropin_loop` leg
puts beside the same loop run through the MI355X drop-ins.

Per episode: reset (a fresh scene on episode 1 and every 200th, main_train.py:79), the first
state's value (main_train.py:87-93), then per step select_action (ppo.py:52-62: the policy's
forward at batch 1, a Categorical sample), env.step (uav_env.py:295-435) and store_transition;
after an episode, update() when the buffer holds >= 4 x BATCH_SIZE transitions (main_train.py:145;
ppo.py:68-181: GAE + normalise, K_EPOCHS epochs of minibatch-64 clipped-PPO Adam steps).
The port: the C oracle env (uav_oracle.c, the reference's recompute-from-scratch algorithm), the
torch-CPU fp32 forward of oracle/policy_ref.py, the numpy GAE of oracle/gae.py, and the torch
autograd + Adam update of uavhip.ppo.ppo_epochs on a CPU module (ppo.py:96-169 restated).

    python -m oracle.cpu_loop_bench --uavs 30 --targets 10 --seconds 8 [--threads 1]

prints one JSON line: env-steps/s over the loop (updates included), the rollout-only rate, and
update() samples/s (transitions per update wall time, 5 epochs)."""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "target-allocation-ppo-transformer_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def run(N, M, seconds, threads):
    import oracle
    from oracle import gae as ogae
    from oracle import policy_ref
    from uavhip.config import Config, params_vector
    from uavhip.policy import TransformerActorCritic
    from uavhip.ppo import make_optimizer, ppo_epochs
    from uavhip.scene import generate_scene
    torch.set_num_threads(threads)
    c = Config()
    c.NUM_UAVS, c.NUM_TARGETS = N, M
    np.random.seed(0)
    random.seed(0)
    torch.manual_seed(0)
    prm = params_vector(c)
    pol = TransformerActorCritic()          # CPU module: the update's parameters
    opt = make_optimizer(pol)
    sd = {k: v.detach() for k, v in pol.state_dict().items()}  # live views for the forward
    env = None
    buf = {"s": [], "a": [], "lp": [], "v": [], "r": [], "d": []}
    st = dict(steps=0, roll_s=0.0, upd_s=0.0, upd_samples=0, updates=0, episodes=0)
    gen = torch.Generator().manual_seed(1)

    def act(state):
        x = torch.from_numpy(state).reshape(1, 5, 14)
        with torch.no_grad():
            logits, value = policy_ref.heads(sd, x)
            p = torch.softmax(logits, -1)[0]
            a = int(torch.multinomial(p, 1, generator=gen).item())
            lp = float(torch.log(p[a]))
        buf["s"].append(x)
        buf["a"].append(a)
        buf["lp"].append(lp)
        buf["v"].append(float(value[0]))
        return a

    def update():
        n = len(buf["a"])
        ret, adv = ogae.gae_1d(buf["r"], buf["d"], buf["v"])
        adv, _, _ = ogae.normalize(adv)
        ppo_epochs(pol, opt, torch.cat(buf["s"]), torch.tensor(buf["a"]), torch.tensor(buf["lp"]),
                   torch.tensor(buf["v"]), torch.from_numpy(ret), torch.from_numpy(adv))
        for k in buf:
            buf[k] = []
        return n

    def episode(i):
        nonlocal env
        if env is None or i == 1 or i % 200 == 0:
            env = oracle.OracleEnv(generate_scene(c), prm)
        state = env.reset()
        with torch.no_grad():
            policy_ref.heads(sd, torch.from_numpy(state).reshape(1, 5, 14))  # Q0 (main_train.py:87-93)
        done, n = False, 0
        while not done:
            a = act(state)
            state, r, done, _ = env.step(a)
            buf["r"].append(r)
            buf["d"].append(done)
            n += 1
        return n

    i = 0
    while True:  # warm-up: up to and including the first update
        i += 1
        episode(i)
        if len(buf["a"]) >= c.BATCH_SIZE * 4:
            update()
            break
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < seconds:
        i += 1
        t0 = time.perf_counter()
        st["steps"] += episode(i)
        st["roll_s"] += time.perf_counter() - t0
        st["episodes"] += 1
        if len(buf["a"]) >= c.BATCH_SIZE * 4:
            t1 = time.perf_counter()
            st["upd_samples"] += update()
            st["upd_s"] += time.perf_counter() - t1
            st["updates"] += 1
    total = time.perf_counter() - t_start
    return {"workload": f"E = 1, {N} UAV x {M} tgt, main_train.py loop", "value": st["steps"] / total,
            "unit": "env-steps/s (loop wall time, updates included)",
            "rollout_env_steps_per_s": st["steps"] / st["roll_s"],
            "update_samples_per_s": st["upd_samples"] / st["upd_s"] if st["upd_s"] > 0 else None,
            "episodes": st["episodes"], "updates": st["updates"], "seconds": total, "cores": threads,
            "kind": "port",
            "sample": (f"{st['episodes']} episodes / {st['steps']} env-steps in {total:.1f} s: C oracle UAVEnv.step + "
                       f"torch-CPU fp32 forward at batch 1 + numpy GAE + torch-CPU autograd/Adam update at "
                       f"minibatch {c.BATCH_SIZE} ({threads} torch thread(s))")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--uavs", type=int, default=30)
    ap.add_argument("--targets", type=int, default=10)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--threads", type=int, default=1)
    a = ap.parse_args()
    print(json.dumps(run(a.uavs, a.targets, a.seconds, a.threads)), flush=True)


if __name__ == "__main__":
    main()
