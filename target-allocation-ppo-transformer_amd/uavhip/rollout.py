"""Batched PPO rollout on one GPU: the hot path of BASELINE.json's north_star.

One iteration = T steps of {fused policy forward -> Philox sample -> fused env step} over E
envs (all on device, no host sync), a bootstrap value pass, GAE + advantage normalisation, and,
with world_size > 1, one all-gather of the trajectory over RCCL. It replaces the
reference's per-transition loop (main_train.py:109-117 -> ppo.py:52-66 -> uav_env.py:295) and its
Python GAE loop (ppo.py:81-89).

Departure from the reference (flagged): the rollout is truncated at a fixed horizon T and the
step after T-1 is bootstrapped with V(s_T) (the reference only ever updates on complete episodes,
main_train.py:140-146, and uses next_value 0 at the buffer end). Pass bootstrap=False for the
reference's rule.
"""
import torch

from . import _lib
from .ppo import gae, gae_workspace


class Trajectory:
    """Device trajectory buffers, time-major [T, E, ...]."""

    def __init__(self, T, E, device, want_info=True):
        f32 = dict(dtype=torch.float32, device=device)
        self.T, self.E = T, E
        self.obs = torch.zeros(T + 1, E, _lib.SEQ_LEN, _lib.STATE_DIM, **f32)  # obs[t] = policy input at t
        self.actions = torch.zeros(T, E, dtype=torch.int8, device=device)
        self.logp = torch.zeros(T, E, **f32)
        self.values = torch.zeros(T, E, **f32)
        self.rewards = torch.zeros(T, E, dtype=torch.float64, device=device)
        self.dones = torch.zeros(T, E, dtype=torch.uint8, device=device)
        self.info = torch.zeros(T, E, _lib.INFO_COUNT, dtype=torch.float64, device=device) if want_info else None
        self.last_values = torch.zeros(E, **f32)
        self.last_actions = torch.zeros(E, dtype=torch.int8, device=device)
        self.last_logp = torch.zeros(E, **f32)
        self.ret, self.adv, self.partials, self.stats = gae_workspace(T, E, device)


class RolloutEngine:
    def __init__(self, env, policy, horizon, want_info=True, bootstrap=True, seed=0):
        self.env = env
        self.policy = policy
        self.T = int(horizon)
        self.bootstrap = bootstrap
        self.seed = int(seed)
        self.traj = Trajectory(self.T, env.E, env.device, want_info)
        self._step_counter = 0

    def start(self, generate=True):
        """Fresh scenes on device (Philox) for every env, episode counter 1, first windows."""
        E = self.env.E
        if generate:
            self.env.istate[:, _lib.IST["EPISODE"]] = 1
            self.env.generate_scenes()
        self.env.reset(episode=1, obs_out=self.traj.obs[0])

    @torch.no_grad()
    def collect(self):
        tr, env, pol = self.traj, self.env, self.policy
        E = env.E
        for t in range(self.T):
            pol.fused_forward(tr.obs[t], action_out=tr.actions[t], logp=tr.logp[t], value=tr.values[t],
                              seed=self.seed, offset=self._step_counter * E)
            self._step_counter += 1
            env.step(tr.actions[t], auto_reset=True, obs_out=tr.obs[t + 1], reward_out=tr.rewards[t],
                     done_out=tr.dones[t], info_out=None if tr.info is None else tr.info[t],
                     want_info=tr.info is not None)
        last = None
        if self.bootstrap:
            pol.fused_forward(tr.obs[self.T], action_out=tr.last_actions, logp=tr.last_logp, value=tr.last_values,
                              seed=self.seed, offset=self._step_counter * E)
            last = tr.last_values
        gae(tr.rewards, tr.dones, tr.values, last_values=last, out=(tr.ret, tr.adv, tr.partials, tr.stats))
        env.refresh_scenes()  # regenerate spare scenes consumed by full resets (off the step path)
        return tr

    def roll(self):
        """Carry the last observation window into the next iteration's obs[0]."""
        self.traj.obs[0].copy_(self.traj.obs[self.T])

    def gather(self, group=None):
        """All-gather the per-rank trajectories over RCCL as one flat fp32 payload per rank
        (uavhip.dist.pack_trajectory); returns the [world * T * E, RECORD_FLOATS] batch."""
        from .dist import all_gather_rows, pack_trajectory
        tr = self.traj
        payload = pack_trajectory(tr.obs[:tr.T], tr.actions, tr.logp, tr.values, tr.ret, tr.adv, tr.rewards,
                                  tr.dones)
        return all_gather_rows(payload, group)
