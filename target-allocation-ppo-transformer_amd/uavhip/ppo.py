"""PPO pieces: the GAE/advantage reduction on the GPU (uavhip_gae + uavhip_adv_normalize) and a
PPOAgent with the reference's API (agents/ppo.py:12-184), used by the drop-in agents/ppo.py.

GAE here follows ppo.py:70-94 op for op in fp32 (returns bit-identical to the reference on the
same buffer); the clipped-PPO epochs (ppo.py:96-181) run on the HIP training step
(uavhip.train.FusedPPOTrainer), or as torch autograd on the GPU (ppo_epochs, GraphPPOUpdater).
"""
import ctypes

import torch
import torch.nn as nn
import torch.optim as optim
from torch.utils.data import BatchSampler, SubsetRandomSampler

from ._lib import LIB, check, ptr, stream_handle
from .config import cfg
from .policy import TransformerActorCritic


def gae(rewards, dones, values, last_values=None, gamma=None, lam=None, normalize=True, out=None):
    """Time-major [T, E] (or 1-D [T]) buffers on the GPU -> (returns, advantages) fp32.

    rewards f64, dones uint8/bool, values f32; last_values [E] f32 bootstraps the step after T-1
    (None = 0, the reference's assumption that the buffer ends on a done, ppo.py:77).
    `advantages` is normalised (ppo.py:94) unless normalize=False; `stats` (mean, std) fp64."""
    gamma = cfg.GAMMA if gamma is None else gamma
    lam = cfg.GAE_LAMBDA if lam is None else lam
    one_d = values.dim() == 1
    T = values.shape[0]
    E = 1 if one_d else values.shape[1]
    dev = values.device
    r = rewards.to(device=dev, dtype=torch.float64).contiguous()
    d = dones.to(device=dev, dtype=torch.uint8).contiguous()
    v = values.to(device=dev, dtype=torch.float32).contiguous()
    lv = None if last_values is None else last_values.to(device=dev, dtype=torch.float32).contiguous()
    if out is None:
        ret = torch.empty_like(v)
        adv = torch.empty_like(v)
        npart = LIB.uavhip_gae_partials(T, E)
        partials = torch.empty(2 * npart, dtype=torch.float64, device=dev)
        stats = torch.empty(2, dtype=torch.float64, device=dev)
    else:
        ret, adv, partials, stats = out
        npart = partials.numel() // 2
    s = stream_handle()
    check(LIB.uavhip_gae(ptr(r), ptr(d), ptr(v), ptr(lv), T, E, ctypes.c_double(gamma), ctypes.c_double(lam),
                         ptr(ret), ptr(adv), ptr(partials), s), "uavhip_gae")
    if normalize:
        check(LIB.uavhip_adv_normalize(ptr(adv), adv.numel(), ptr(partials), npart, 0, ptr(stats), s),
              "uavhip_adv_normalize")
    return ret, adv, stats


def gae_workspace(T, E, device):
    npart = LIB.uavhip_gae_partials(T, E)
    return (torch.empty(T, E, dtype=torch.float32, device=device), torch.empty(T, E, dtype=torch.float32, device=device),
            torch.empty(2 * npart, dtype=torch.float64, device=device), torch.empty(2, dtype=torch.float64, device=device))


def ppo_epochs(policy, optimizer, states, actions, old_logprobs, old_values, returns, advantages, epochs=None,
               batch_size=None, eps_clip=None, grad_clip=None, generator=None, perms=None, on_step=None):
    """Clipped-PPO minibatch epochs (ppo.py:96-169). Returns (mean actor loss, critic loss, entropy, n).
    Minibatches: BatchSampler(SubsetRandomSampler(range(n), generator), batch_size, drop_last=True)
    per epoch as ppo.py:115, or over the given per-epoch row orders `perms` (recorded sampler draws).
    on_step(): called after every optimizer step (tests record the optimizer state)."""
    epochs = cfg.K_EPOCHS if epochs is None else epochs
    batch_size = cfg.BATCH_SIZE if batch_size is None else batch_size
    eps = cfg.EPS_CLIP if eps_clip is None else eps_clip
    gclip = cfg.GRAD_NORM_CLIP if grad_clip is None else grad_clip
    mse = nn.MSELoss()
    n = states.shape[0]
    dev = states.device
    sa = sc = se = 0.0
    cnt = 0
    acc = torch.zeros(3, dtype=torch.float64, device=dev)
    if perms is not None:
        epochs = len(perms)
    for ep in range(epochs):
        order = [int(i) for i in perms[ep]] if perms is not None else \
            SubsetRandomSampler(range(n), generator=generator)
        for idx in BatchSampler(order, batch_size, drop_last=True):
            idx = torch.as_tensor(idx, device=dev)
            logp, v, ent = policy.evaluate(states[idx], actions[idx])
            v = torch.squeeze(v)
            ratios = torch.exp(logp - old_logprobs[idx])
            adv = advantages[idx]
            surr1 = ratios * adv
            surr2 = torch.clamp(ratios, 1 - eps, 1 + eps) * adv
            loss_actor = -torch.min(surr1, surr2).mean()
            bov = old_values[idx]
            v_clip = bov + torch.clamp(v - bov, -eps, eps)
            loss_critic = torch.max(mse(v, returns[idx]), mse(v_clip, returns[idx]))
            ent_mean = ent.mean()
            loss = loss_actor + 0.5 * loss_critic - 0.01 * ent_mean
            optimizer.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(policy.parameters(), gclip)
            acc += torch.stack([loss_actor.detach(), loss_critic.detach(), ent_mean.detach()]).double()
            cnt += 1
            optimizer.step()
            if on_step is not None:
                on_step()
    if cnt:
        sa, sc, se = (acc / cnt).tolist()
    return sa, sc, se, cnt


def make_optimizer(policy, capturable=False):
    """Adam with the reference's four parameter groups (ppo.py:17-22); capturable=True keeps the
    step counters on device so the step can live in a captured graph (GraphPPOUpdater)."""
    groups = [
        {"params": policy.actor_head.parameters(), "lr": cfg.LR_ACTOR},
        {"params": policy.actor_net.parameters(), "lr": cfg.LR_ACTOR},
        {"params": policy.critic_head.parameters(), "lr": cfg.LR_CRITIC},
        {"params": policy.critic_net.parameters(), "lr": cfg.LR_CRITIC},
    ]
    if capturable:
        return optim.Adam(groups, capturable=True, foreach=True)
    return optim.Adam(groups)


class PPOAgent:
    """agents/ppo.py:12-184 API: select_action / store_transition / update / clear_buffer,
    attributes device, policy, policy_old, optimizer, buffer, mse_loss."""

    def __init__(self, fused_update=True):
        """fused_update: update() runs the HIP training step (uavhip.train.FusedPPOTrainer, its own
        Adam moments in `self.trainer`); False runs ppo_epochs with torch autograd + self.optimizer."""
        if not torch.cuda.is_available():
            raise RuntimeError("PPOAgent (uavhip) needs an MI355X: the rollout forward is a HIP kernel")
        self.device = torch.device("cuda")
        self.policy = TransformerActorCritic().to(self.device)
        self.optimizer = make_optimizer(self.policy)
        self.fused_update = bool(fused_update) and cfg.BATCH_SIZE % 64 == 0
        self.trainer = None
        self.policy_old = TransformerActorCritic().to(self.device)
        self.policy_old.load_state_dict(self.policy.state_dict())
        self.buffer = {"states": [], "actions": [], "logprobs": [], "rewards": [], "is_terminals": [], "values": []}
        self.mse_loss = nn.MSELoss()

    def select_action(self, state):
        x = torch.as_tensor(state, dtype=torch.float32).reshape(1, cfg.SEQ_LEN, cfg.STATE_DIM).to(self.device)
        action, logp, value, _ = self.policy_old.get_action(x)
        self.buffer["states"].append(x)
        self.buffer["actions"].append(action)
        self.buffer["logprobs"].append(logp)
        self.buffer["values"].append(value)
        # one device->host copy (the sync the reference's loop already has): the action and a finite flag
        ok = torch.isfinite(logp).all() & torch.isfinite(value).all()
        host = torch.stack([action.reshape(-1)[0].to(torch.float32), ok.to(torch.float32)]).cpu()
        a = int(host[0])
        if not bool(host[1]):
            # torch's Categorical rejects non-finite probabilities (transformer_net.py:118-120); here
            # they mean a split-product operand left fp16's range (|x| >= 65536, common.hpp f16_lo)
            raise ValueError("the policy produced a non-finite log-probability / value (an activation beyond "
                             "the split products' fp16 range)")
        return a

    def store_transition(self, reward, done):
        self.buffer["rewards"].append(reward)
        self.buffer["is_terminals"].append(done)

    def update(self):
        if not self.buffer["values"]:
            self.clear_buffer()
            return None
        values = torch.cat(self.buffer["values"], dim=0).reshape(-1)
        rewards = torch.tensor(self.buffer["rewards"], dtype=torch.float64)
        dones = torch.tensor([bool(d) for d in self.buffer["is_terminals"]], dtype=torch.uint8)
        returns, advantages, _ = gae(rewards, dones, values)
        old_states = torch.cat(self.buffer["states"], dim=0)
        old_actions = torch.cat(self.buffer["actions"], dim=0)
        old_logprobs = torch.cat(self.buffer["logprobs"], dim=0)
        if self.fused_update:
            from .train import FusedPPOTrainer
            if self.trainer is None:
                self.trainer = FusedPPOTrainer(self.policy, cfg.BATCH_SIZE)
            # the trainer's own buffers (fixed addresses): one captured hipGraph per epoch length,
            # reused by every later update with the same number of minibatches
            self.trainer.stage(old_states, old_actions, old_logprobs, values.detach(), returns, advantages)
            sa, sc, se, cnt = self.trainer.run(use_graph=True)
        else:
            sa, sc, se, cnt = ppo_epochs(self.policy, self.optimizer, old_states, old_actions, old_logprobs,
                                         values.detach(), returns, advantages)
        self.policy_old.load_state_dict(self.policy.state_dict())
        self.clear_buffer()
        if cnt == 0:
            return None
        return {"loss_actor": sa, "loss_critic": sc, "entropy": se}

    def clear_buffer(self):
        self.buffer = {k: [] for k in self.buffer}


class GraphPPOUpdater:
    """The clipped-PPO minibatch step of ppo_epochs (ppo.py:96-169), captured once into a hipGraph
    and replayed per minibatch: evaluate -> losses -> backward -> clip_grad_norm_ -> Adam, with the
    minibatch gathered on device from the (fixed) trajectory buffers by a static index tensor.

    Same ops and op order as ppo_epochs on the same minibatch order (torch.randperm of the CPU
    generator, SubsetRandomSampler's draw), so a replay reproduces an eager step up to atomics in
    the backward kernels. The optimizer must be Adam built with capturable=True (make_optimizer(
    policy, capturable=True)). Buffers must keep their storage for the updater's lifetime."""

    def __init__(self, policy, optimizer, states, actions, old_logprobs, old_values, returns, advantages,
                 batch_size, eps_clip=None, grad_clip=None):
        self.policy, self.opt = policy, optimizer
        self.bufs = (states, actions, old_logprobs, old_values, returns, advantages)
        self.n = states.shape[0]
        self.bs = int(batch_size)
        self.eps = cfg.EPS_CLIP if eps_clip is None else eps_clip
        self.gclip = cfg.GRAD_NORM_CLIP if grad_clip is None else grad_clip
        dev = states.device
        self.idx = torch.zeros(self.bs, dtype=torch.long, device=dev)
        self.acc = torch.zeros(3, dtype=torch.float64, device=dev)
        self.graph = None

    def _step(self):
        states, actions, old_logprobs, old_values, returns, advantages = self.bufs
        idx, eps = self.idx, self.eps
        logp, v, ent = self.policy.evaluate(states[idx], actions[idx], validate=False)
        v = torch.squeeze(v)
        ratios = torch.exp(logp - old_logprobs[idx])
        adv = advantages[idx]
        surr1 = ratios * adv
        surr2 = torch.clamp(ratios, 1 - eps, 1 + eps) * adv
        loss_actor = -torch.min(surr1, surr2).mean()
        bov = old_values[idx]
        ret = returns[idx]
        v_clip = bov + torch.clamp(v - bov, -eps, eps)
        loss_critic = torch.max(torch.mean((v - ret) ** 2), torch.mean((v_clip - ret) ** 2))
        ent_mean = ent.mean()
        loss = loss_actor + 0.5 * loss_critic - 0.01 * ent_mean
        self.opt.zero_grad(set_to_none=False)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(self.policy.parameters(), self.gclip)
        self.acc += torch.stack([loss_actor.detach(), loss_critic.detach(), ent_mean.detach()]).double()
        self.opt.step()

    def capture(self, warmup=2):
        """Warm up (allocates grads / optimizer state) on a side stream, then capture one step."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        snapshot = [p.detach().clone() for p in self.policy.parameters()]
        opt_state = {k: {kk: (vv.clone() if torch.is_tensor(vv) else vv) for kk, vv in st.items()}
                     for k, st in self.opt.state.items()}
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._step()
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._step()
        # undo the warm-up / capture side effects on weights and optimizer state
        with torch.no_grad():
            for p, q in zip(self.policy.parameters(), snapshot):
                p.copy_(q)
            for p, st in self.opt.state.items():
                old = opt_state.get(p)
                for k, v in st.items():
                    if torch.is_tensor(v):
                        if old is not None and k in old:
                            v.copy_(old[k])
                        else:
                            v.zero_()
        self.acc.zero_()

    def run(self, epochs=None, generator=None):
        """K epochs over the buffers -> (mean actor loss, critic loss, entropy, n_steps)."""
        epochs = cfg.K_EPOCHS if epochs is None else epochs
        if self.graph is None:
            self.capture()
        self.acc.zero_()
        cnt = 0
        for _ in range(epochs):
            perm = torch.randperm(self.n, generator=generator).to(self.idx.device, non_blocking=True)
            for b in range(self.n // self.bs):
                self.idx.copy_(perm[b * self.bs:(b + 1) * self.bs])
                self.graph.replay()
                cnt += 1
        if cnt == 0:
            return 0.0, 0.0, 0.0, 0
        sa, sc, se = (self.acc / cnt).tolist()
        return sa, sc, se, cnt
