"""Batched PPO rollout on one GPU: the hot path of BASELINE.json's north_star.

One iteration = T steps of {fused policy forward -> Philox sample -> fused env step} over E
envs (all on device, no host sync), a bootstrap value pass, GAE + advantage normalisation, the
refresh of spare scenes consumed by full resets, and (caller) with world_size > 1 one all-gather
of the trajectory over RCCL. It replaces the reference's per-transition loop
(main_train.py:109-117 -> ppo.py:52-66 -> uav_env.py:295) and its Python GAE loop (ppo.py:81-89).

The iteration can be captured once into a hipGraph (`capture()`) and replayed: the sampling
counter then lives on the device (advanced by the graph itself), and the policy weights are
repacked in place, so replays stay valid across PPO updates.

Departure from the reference (flagged): the rollout is truncated at a fixed horizon T and the
step after T-1 is bootstrapped with V(s_T) (the reference only ever updates on complete episodes,
main_train.py:140-146, and uses next_value 0 at the buffer end). Pass bootstrap=False for the
reference's rule.
"""
import os

import torch

from . import _lib
from .policy import rowproj_buffer
from .ppo import gae, gae_workspace

# UAVHIP_BOOTSTRAP_FULL=1: the bootstrap V(s_T) through the full forward (actor + sampling + critic)
# instead of the critic-only launch -- the same values, bitwise (A/B switch of scripts/gpu_r04z.sh)
_BOOTSTRAP_FULL = os.environ.get("UAVHIP_BOOTSTRAP_FULL", "0") == "1"


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
        self.last_values = torch.zeros(E, **f32)  # V(s_T), the bootstrap
        self.ret, self.adv, self.partials, self.stats = gae_workspace(T, E, device)


class RolloutEngine:
    def __init__(self, env, policy, horizon, want_info=True, bootstrap=True, seed=None, normalize=True, row_cache=True,
                 fused_step=None, total_envs=None, persistent=None, group=None):
        """normalize=False leaves the advantages raw after GAE: a data-parallel caller normalises
        them with the moments of the whole data-parallel batch in normalize_global() (called by
        gather()) (ppo.py:94).
        row_cache=False runs every step on the full-window forward (uavhip_policy_forward).
        fused_step: one launch per step (uavhip_rollout_step: forward + sample + env step); default
        on when the row cache is on and N, M <= 64.
        persistent: the T fused steps of an iteration as ONE launch (uavhip_rollout_steps: every
        workgroup loops over the steps of its own envs); default on with fused_step and f32
        observations. Bitwise the same trajectory as T uavhip_rollout_step launches.
        seed: Philox key of the action sampling (default: the policy's sample_seed, drawn from
        torch's RNG). Sampling counters are global env indices: step t of env e draws counter
        t * total_envs + env.env_base + e, so a rank's shard (VecUAVEnv(env_base=shard start),
        total_envs = all ranks' envs, the same seed everywhere) samples exactly what the same envs
        sample in one process over the union, and no two ranks share a counter.
        group: the torch.distributed process group of the data-parallel rollout (default: WORLD).
        Construction is COLLECTIVE over it when torch.distributed is initialised (resolve_shards
        all-gathers every rank's env block): build the engine on every rank of `group` at the same
        point; normalize_global / gather / gather_submit use the same group by default."""
        self.env = env
        self.normalize = normalize
        self.iteration = 0
        self._gathered = (-1, None, None)  # (iteration, batch, pending event) of the last gather()
        self._submitted = -1  # iteration of the payload gather_submit() enqueued
        self._normalized = -1        # iteration whose advantages normalize_global() normalised
        self.policy = policy
        self.T = int(horizon)
        self.bootstrap = bootstrap
        self.seed = int(policy.sample_seed if seed is None else seed)
        self.env_base = int(getattr(env, "env_base", 0))
        # world > 1: the ranks' env blocks are all-gathered and checked (disjoint, tiling total), and
        # total defaults to their sum -- the sampling counters and the global advantage count use it
        from .dist import resolve_shards
        self.group = group
        self.total = resolve_shards(env.E, self.env_base, total_envs, group=group, device=env.device)
        self.traj = Trajectory(self.T, env.E, env.device, want_info)
        self.counter = torch.zeros(1, dtype=torch.int64, device=env.device)  # sampling counter base
        # window-row projections of the obs windows (policy.rowproj_buffer): the windows of one
        # iteration are one deque sequence, so step t projects only its new row (rebuilt at t = 0)
        self.rowproj = rowproj_buffer(env.E, env.device) if row_cache else None
        can_fuse = row_cache and env.N <= 64 and env.M <= 64
        if fused_step and not can_fuse:
            raise ValueError("fused_step needs row_cache=True and N, M <= 64")
        self.fused_step = can_fuse if fused_step is None else bool(fused_step)
        can_persist = self.fused_step and env.obs_dtype == torch.float32
        if persistent and not can_persist:
            raise ValueError("persistent needs fused_step and float32 observations")
        self.persistent = can_persist if persistent is None else bool(persistent)
        self.graph = None
        self.policy_events = None   # [(start, end)] HIP events around each policy launch (optional)
        self.env_events = None

    def start(self, generate=True):
        """Fresh scenes on device (Philox) for every env, episode counter 1, first windows."""
        if generate:
            self.env.istate[:, _lib.IST["EPISODE"]] = 1
            self.env.generate_scenes()
        self.env.reset(episode=1, obs_out=self.traj.obs[self.T])  # moved to obs[0] by the first _body

    def _offset(self, t):
        """Sampling counter base of step t (the device counter adds (T + 1) * total per iteration)."""
        return t * self.total + self.env_base

    def _forward(self, t, obs, actions, logp, value):
        ev = self.policy_events
        if ev is not None:
            ev[t][0].record()
        self.policy.fused_forward(obs, action_out=actions, logp=logp, value=value, seed=self.seed,
                                  offset=self._offset(t), offset_dev=self.counter, check_weights=False,
                                  rowproj=self.rowproj, step=t, fill=t == 0)
        if ev is not None:
            ev[t][1].record()

    def _body(self):
        tr, env = self.traj, self.env
        tr.obs[0].copy_(tr.obs[self.T])  # carry the previous iteration's last window
        eev = self.env_events
        if self.persistent:  # the whole horizon in one launch; step t is the same as in the loop below
            ev = self.policy_events
            if ev is not None:
                ev[0][0].record()
            self.policy.rollout_steps(env, tr.obs, self.rowproj, 0, True, tr.actions, tr.logp, tr.values,
                                      tr.rewards, tr.dones, tr.info, seed=self.seed, offset=self._offset(0),
                                      offset_stride=self.total, offset_dev=self.counter)
            if ev is not None:
                ev[0][1].record()
        for t in range(0 if self.persistent else self.T):
            if self.fused_step:
                ev = self.policy_events
                if ev is not None:
                    ev[t][0].record()
                self.policy.rollout_step(env, tr.obs[t], self.rowproj, t, t == 0, tr.actions[t], tr.logp[t],
                                         tr.values[t], tr.obs[t + 1], tr.rewards[t], tr.dones[t],
                                         None if tr.info is None else tr.info[t], seed=self.seed,
                                         offset=self._offset(t), offset_dev=self.counter)
                if ev is not None:
                    ev[t][1].record()
                continue
            self._forward(t, tr.obs[t], tr.actions[t], tr.logp[t], tr.values[t])
            if eev is not None:
                eev[t][0].record()
            env.step(tr.actions[t], auto_reset=True, obs_out=tr.obs[t + 1], reward_out=tr.rewards[t],
                     done_out=tr.dones[t], info_out=None if tr.info is None else tr.info[t],
                     want_info=tr.info is not None)
            if eev is not None:
                eev[t][1].record()
        last = None
        if self.bootstrap:
            if self.rowproj is not None and not _BOOTSTRAP_FULL:
                # the critic alone (uavhip_policy_value_rows): nothing reads an action at step T; the
                # actor ring row it skips is rebuilt by the next iteration's fill (step 0, fill=True)
                ev = self.policy_events
                if ev is not None:
                    ev[self.T][0].record()
                self.policy.value_rows(tr.obs[self.T], self.rowproj, self.T, tr.last_values)
                if ev is not None:
                    ev[self.T][1].record()
            else:
                self._forward(self.T, tr.obs[self.T], None, None, tr.last_values)
            last = tr.last_values
        gae(tr.rewards, tr.dones, tr.values, last_values=last, normalize=self.normalize,
            out=(tr.ret, tr.adv, tr.partials, tr.stats))
        env.refresh_scenes()  # regenerate spare scenes consumed by full resets (off the step path)
        self.counter.add_((self.T + 1) * self.total)

    @torch.no_grad()
    def collect(self, eager=False):
        """One rollout iteration: a graph replay when captured (unless eager=True), else eager
        launches (which also record the HIP events, if enabled). Both advance the same device state."""
        self.policy.packed_weights()  # repack in place if the weights changed (e.g. after an update)
        self.iteration += 1
        if self.graph is not None and not eager:
            self.graph.replay()
        else:
            self._body()
        return self.traj

    def check_finite(self):
        """Raise if the last iteration's log-probabilities or values are not finite (one reduction and
        a host sync; not called by collect()). Non-finite policy outputs are how the split-product
        forward flags an activation beyond fp16's range (|x| >= 65536, common.hpp f16_lo): never a
        finite wrong value."""
        tr = self.traj
        ok = torch.isfinite(tr.logp).all() & torch.isfinite(tr.values).all()
        if not bool(ok):
            raise FloatingPointError("rollout: non-finite log-probabilities / values (an activation beyond the "
                                     "split products' fp16 range)")
        return True

    def roll(self):
        """Kept for API compatibility: each iteration starts by carrying obs[T] into obs[0]."""

    def enable_events(self, external=False):
        """HIP events around every policy / env launch (external=True: graph-capturable nodes)."""
        kw = dict(enable_timing=True)
        if external:
            kw["external"] = True
        self.policy_events = [(torch.cuda.Event(**kw), torch.cuda.Event(**kw)) for _ in range(self.T + 1)]
        self.env_events = [(torch.cuda.Event(**kw), torch.cuda.Event(**kw)) for _ in range(self.T)]

    def event_ms(self):
        """(policy launch ms list, env launch ms list) of the most recent iteration (fused steps:
        the policy list holds the T fused launches + the bootstrap forward, the env list is empty)."""
        if self.persistent:  # one launch of T steps: its per-step average T times, then the bootstrap
            one = self.policy_events[0][0].elapsed_time(self.policy_events[0][1]) / self.T
            a, b = self.policy_events[self.T]
            return [one] * self.T + ([a.elapsed_time(b)] if self.bootstrap else []), []
        pol = [a.elapsed_time(b) for a, b in self.policy_events]
        env = [] if self.fused_step else [a.elapsed_time(b) for a, b in self.env_events]
        return pol, env

    @torch.no_grad()
    def capture(self):
        """Capture one iteration into a hipGraph. The state it advances lives on the device,
        so every replay is the next iteration. HIP events are not captured (ROCm disallows
        external events in graphs); eager iterations still record them."""
        events = (self.policy_events, self.env_events)
        self.policy_events = self.env_events = None
        self.policy.packed_weights()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up outside capture (allocator / lazy init)
            self._body()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._body()
        self.graph = g
        self.policy_events, self.env_events = events
        return g

    def normalize_global(self, group=None):
        """The data-parallel exchange the update on set_shard() batches needs: a
        3-double all-reduce of the advantage moments and normalisation of this rank's advantages
        with them (ppo.py:94 normalises over the whole batch). Once per iteration; a no-op when the
        engine normalised locally (one rank)."""
        from .dist import global_moments, normalize_global
        group = self.group if group is None else group
        if self.normalize or self._normalized == self.iteration:
            return self.traj
        tr = self.traj
        normalize_global(tr.adv, global_moments(tr.partials, tr.adv.numel(), group), count=self.T * self.total)
        self._normalized = self.iteration
        return tr

    def gather(self, group=None):
        """The data-parallel exchange of one iteration: a 3-double all-reduce of the
        advantage moments and normalisation with them (when the engine left the advantages raw),
        then ONE all-gather over RCCL of every rank's compact payload (uavhip.dist.pack_compact:
        20 floats per transition) and the GPU rebuild of the windows. Returns the gathered batch
        as a dict of [world * T * E, ...] tensors (obs, actions, logp, values, returns, advantages,
        dones) in (rank, step, env) order."""
        from .dist import all_gather_rows, pack_compact, unpack_compact
        group = self.group if group is None else group
        if self._gathered[0] == self.iteration:  # once per iteration (normalises in place)
            batch, ev = self._gathered[1], self._gathered[2]
            if ev is not None:  # from the pipelined exchange: complete on its side stream
                cur = torch.cuda.current_stream()
                cur.wait_event(ev)
                for t in batch.values():
                    t.record_stream(cur)
                self._gathered = (self.iteration, batch, None)
            return batch
        tr = self.normalize_global(group)
        payload = pack_compact(tr.obs, tr.actions, tr.logp, tr.values, tr.ret, tr.adv, tr.dones)
        gathered = all_gather_rows(payload.view(1, -1), group)
        batch = unpack_compact(gathered, tr.T, tr.E)
        self._gathered = (self.iteration, batch, None)
        return batch

    def gather_submit(self, exchange, group=None):
        """The pipelined form of gather() (uavhip.dist.IpcAllGather): normalise with the global moments
        and enqueue this iteration's compact payload; gather_finish() completes the exchange -- call
        it after enqueueing the next iteration's rollout, beside which the copies then run."""
        from .dist import pack_compact
        tr = self.normalize_global(self.group if group is None else group)
        exchange.submit(pack_compact(tr.obs, tr.actions, tr.logp, tr.values, tr.ret, tr.adv, tr.dones))
        self._submitted = self.iteration

    def gather_finish(self, exchange):
        """Complete the submitted exchange: the peer copies and the window rebuild on the exchange's
        side stream. The batch (as gather() returns it) is what gather() returns while no later
        iteration has been collected; its consumers wait on the returned event."""
        from .dist import unpack_compact
        recv, ev = exchange.progress()
        side = exchange.side
        with torch.cuda.stream(side):
            # scalars copied out of the receive buffer: progress() rewrites it two iterations later
            # without waiting for this batch's consumers
            batch = unpack_compact(recv, self.T, self.env.E, copy=True)
        done = torch.cuda.Event()
        done.record(side)
        if self._submitted == self.iteration:
            self._gathered = (self.iteration, batch, done)
        return batch, done
