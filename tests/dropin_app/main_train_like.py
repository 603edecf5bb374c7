"""The reference's training driver (main_train.py:35-238) restated for the drop-in GPU test: the
same imports, the same loop over UAVEnv / PPOAgent (Q0 from policy_old.get_action, select_action ->
env.step -> store_transition, update once the buffer holds 4 x BATCH_SIZE transitions, the
per-episode statistics and the CSV every 10 episodes, state_dict checkpoints), minus matplotlib's
learning curve. Run through `python -m uavhip.run_reference main_train_like.py --episodes N`; it
prints one JSON summary line. Test infrastructure (tests/test_gpu_dropin.py)."""
import argparse
import csv
import json
import os
import sys

import numpy as np
import torch

from configs.config import cfg
from envs.uav_env import UAVEnv
from agents.ppo import PPOAgent


def train(episodes):
    env = UAVEnv()
    agent = PPOAgent()
    os.makedirs("logs", exist_ok=True)
    os.makedirs("saved_models", exist_ok=True)
    csv_file = open(os.path.join("logs", "training_stats.csv"), mode="w", newline="", encoding="utf-8")
    writer = csv.writer(csv_file)
    writer.writerow(["Episode", "Avg_Reward", "Avg_Q0", "Avg_J_Value", "Max_Coverage", "Action1_Ratio",
                     "Valid_Assign_Rate", "Avg_P_Dmg", "Avg_P_Final", "Loss_Critic", "Loss_Actor", "Entropy"])
    ep_rewards, ep_q0s, updates, steps_total, last_stats = [], [], 0, 0, None
    for i_episode in range(1, episodes + 1):
        state = env.reset(full_reset=(i_episode == 1 or i_episode % 200 == 0))
        current_ep_reward = 0
        done = False
        with torch.no_grad():
            _, _, q0_val, _ = agent.policy_old.get_action(torch.FloatTensor(state).unsqueeze(0).to(agent.device))
            current_q0 = q0_val.item()
        ep_total_J, ep_steps, ep_max_cov, ep_action1_cnt, ep_valid_cnt = 0, 0, 0, 0, 0
        ep_total_p_dmg, ep_total_p_final, ep_steps_with_assign = 0.0, 0.0, 0
        while not done:
            action = agent.select_action(state)
            next_state, reward, done, info = env.step(action)
            agent.store_transition(reward, done)
            state = next_state
            current_ep_reward += reward
            ep_steps += 1
            if info:
                ep_total_J += info.get("J_val", 0)
                ep_max_cov = max(ep_max_cov, info.get("num_assigned", 0))
                if action == 1:
                    ep_action1_cnt += 1
                    if info.get("is_valid_action", False):
                        ep_valid_cnt += 1
                if info.get("num_assigned", 0) > 0:
                    ep_total_p_dmg += info.get("avg_p_dmg", 0)
                    ep_total_p_final += info.get("avg_p_final", 0)
                    ep_steps_with_assign += 1
        steps_total += ep_steps
        ppo_stats = None
        if len(agent.buffer["states"]) >= cfg.BATCH_SIZE * 4:
            ppo_stats = agent.update()
            updates += 1
            last_stats = ppo_stats
        ep_rewards.append(current_ep_reward)
        ep_q0s.append(current_q0)
        if i_episode % 10 == 0:
            l_crt = ppo_stats["loss_critic"] if ppo_stats else 0.0
            l_act = ppo_stats["loss_actor"] if ppo_stats else 0.0
            entr = ppo_stats["entropy"] if ppo_stats else 0.0
            writer.writerow([i_episode, f"{np.mean(ep_rewards[-50:]):.4f}", f"{np.mean(ep_q0s[-50:]):.4f}",
                             f"{ep_total_J / max(1, ep_steps):.4f}", ep_max_cov,
                             f"{ep_action1_cnt / max(1, ep_steps):.4f}", f"{ep_valid_cnt / max(1, ep_action1_cnt):.4f}",
                             f"{ep_total_p_dmg / max(1, ep_steps_with_assign):.4f}",
                             f"{ep_total_p_final / max(1, ep_steps_with_assign):.4f}",
                             f"{l_crt:.6f}", f"{l_act:.6f}", f"{entr:.6f}"])
            csv_file.flush()
        torch.save(agent.policy.state_dict(), os.path.join("saved_models", "final_model.pth"))
    csv_file.close()
    mods = {m: sys.modules[m].__file__ for m in ("configs.config", "envs.uav_env", "envs.entities", "agents.ppo")}
    return {"episodes": episodes, "updates": updates, "steps": steps_total, "last_stats": last_stats,
            "rewards": [float(r) for r in ep_rewards], "modules": mods}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=20)
    args = ap.parse_args()
    print(json.dumps(train(args.episodes)), flush=True)
