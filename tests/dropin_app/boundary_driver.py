"""Drop-in harness for tests/test_gpu_dropin.py: exercises the Python surface that SURVEY.md 8(b)
lists as the boundary -- what the reference's driver (main_train.py:41-42, 79, 87-93, 111-117,
145-146, 211, 232) calls on the env and the agent -- through the launcher
`python -m uavhip.run_reference main_train.py --episodes N`, and prints one JSON report.

Contract checked:
  UAVEnv(); reset(full_reset) -> float32 [5, 14]; step(int) -> (obs [5, 14] or [14] when done,
  float reward, bool done, info with J_val / num_assigned / is_valid_action / avg_p_dmg / avg_p_final);
  PPOAgent(); .device; .policy_old.get_action(x) -> (action, logp, value, entropy);
  .select_action(state) -> int; .store_transition(reward, done); .buffer['states'] (its length gates
  the update); .update() -> {loss_actor, loss_critic, entropy} or None; .policy.state_dict().
The per-episode statistics main_train derives from `info` are pinned separately by the
tests/golden/main_train.npz fixture (tests/test_gpu_metrics.py); this harness only drives the calls.
Test infrastructure only."""
import argparse
import json
import os
import sys

import torch

from configs.config import cfg
from envs.uav_env import UAVEnv
from agents.ppo import PPOAgent

INFO_KEYS = {"J_val", "num_assigned", "is_valid_action", "avg_p_dmg", "avg_p_final"}


class Probe:
    """Counts what the boundary returned and checks its types as it goes."""

    def __init__(self):
        self.steps = self.updates = self.episodes = 0
        self.returns, self.losses, self.terminal_shapes = [], [], set()

    def check_step(self, action, out):
        obs, reward, done, info = out
        assert isinstance(reward, float) and isinstance(done, bool), (type(reward), type(done))
        assert INFO_KEYS <= set(info), sorted(info)
        assert isinstance(info["num_assigned"], int)
        assert info["is_valid_action"] is None if action == 0 else isinstance(info["is_valid_action"], bool)
        if done:
            self.terminal_shapes.add(tuple(obs.shape))
        else:
            assert obs.shape == (cfg.SEQ_LEN, cfg.STATE_DIM) and str(obs.dtype) == "float32"
        self.steps += 1


def run_episode(env, agent, probe, episode):
    # the reference resets the scene on the first episode and every 200th (main_train.py:79)
    state = env.reset(full_reset=episode == 1 or episode % 200 == 0)
    assert state.shape == (cfg.SEQ_LEN, cfg.STATE_DIM)
    with torch.no_grad():  # the value of the first state (main_train.py:87-93)
        out = agent.policy_old.get_action(torch.as_tensor(state).unsqueeze(0).to(agent.device))
        assert len(out) == 4
    total, done = 0.0, False
    while not done:
        action = agent.select_action(state)
        assert action in (0, 1)
        res = env.step(action)
        probe.check_step(action, res)
        state, reward, done, _ = res
        agent.store_transition(reward, done)
        total += reward
    probe.returns.append(total)
    probe.episodes += 1


def main(episodes):
    env, agent, probe = UAVEnv(), PPOAgent(), Probe()
    os.makedirs("saved_models", exist_ok=True)
    for episode in range(1, episodes + 1):
        run_episode(env, agent, probe, episode)
        if len(agent.buffer["states"]) >= cfg.BATCH_SIZE * 4:  # the update gate (main_train.py:145)
            stats = agent.update()
            assert stats is None or set(stats) == {"loss_actor", "loss_critic", "entropy"}
            assert len(agent.buffer["states"]) == 0
            probe.updates += 1
            probe.losses.append(stats)
    path = os.path.join("saved_models", "final_model.pth")
    torch.save(agent.policy.state_dict(), path)
    mods = {m: sys.modules[m].__file__ for m in ("configs.config", "envs.uav_env", "envs.entities", "agents.ppo")}
    return {"episodes": probe.episodes, "updates": probe.updates, "steps": probe.steps,
            "last_stats": probe.losses[-1] if probe.losses else None, "rewards": probe.returns,
            "terminal_shapes": sorted(probe.terminal_shapes), "modules": mods, "checkpoint": path}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=20)
    print(json.dumps(main(ap.parse_args().episodes)), flush=True)
