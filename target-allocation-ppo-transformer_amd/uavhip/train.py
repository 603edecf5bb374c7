"""FusedPPOTrainer: the clipped-PPO update of agents/ppo.py:96-169 on the HIP training step of
libuavhip.so (uavhip_ppo_step, csrc/train.hip) -- fp32-accurate split-product GEMMs on the f16 MFMA
(forward and input gradients two-plane, weight gradients three-plane; gradients carried pre-scaled
by the power of two >= the minibatch so the planes stay in fp16's normal range), fused LayerNorm /
attention / heads+loss kernels and a fused clip_grad_norm_ + Adam.

The policy's parameters become views of one flat buffer (the uavhip_policy_layout() order), so
state_dict(), load_state_dict() and the torch `evaluate` path keep working on the same storage the
kernels update. One minibatch step is one C call; `run` captures the steps of a whole epoch into
one hipGraph (minibatch b reads its rows at a fixed offset of a device permutation buffer) and per
epoch copies in the permutation and replays it, drawing minibatches like SubsetRandomSampler
(torch.randperm of the given CPU generator, ppo.py:97-99).

Data parallel (world > 1, the same generator seed on every rank), two ways to hold the batch:
  * set_shard (the default data path, no trajectory exchange): every rank keeps its own rollout
    shard; minibatches are drawn over the world * n_local global rows exactly as on one GPU, and
    each rank computes the rows of every global minibatch that it owns (a varying count, padded with
    idx -1 rows to a multiple of 64);
  * set_buffers on all-gathered buffers (RolloutEngine.gather): each rank takes its 1/world slice of
    every global minibatch.
Either way one step is FORWARD, an all-reduce of the four loss sums (the clipped value loss picks
max(...) over the GLOBAL minibatch), BACKWARD (gradients scaled by 1/global minibatch), an
all-reduce of the flat gradient (1.68 MB over RCCL/xGMI), then the same clip + Adam on every rank:
the result is the single-GPU step on the global minibatch (fp32 sums in another order). On an RCCL
group ("nccl") the collectives are captured with the kernels: a data-parallel epoch over gathered
buffers is one hipGraph replay like a single-GPU one (gloo's collectives run on the host: eager).
"""
import ctypes

import torch

from . import _lib
from ._lib import LIB, check, ptr, stream_handle
from .config import cfg
from .policy import layout


class FusedPPOTrainer:
    def __init__(self, policy, minibatch, lr_actor=None, lr_critic=None, eps_clip=None, max_grad_norm=None,
                 value_coef=0.5, entropy_coef=0.01, betas=(0.9, 0.999), adam_eps=1e-8, world=None, rank=None,
                 group=None, allreduce=None, data_parallel=None):
        """minibatch: samples per optimizer step over all ranks (each rank runs minibatch / world).
        world / rank default to torch.distributed's (1 / 0 when not initialised); allreduce(t)
        sums a device tensor over the ranks in place (default: torch.distributed.all_reduce).
        data_parallel: run the phase-split step with its two all-reduces (default: world > 1)."""
        import torch.distributed as tdist
        ddp = tdist.is_available() and tdist.is_initialized()
        self.world = int(world if world is not None else (tdist.get_world_size(group) if ddp else 1))
        self.rank = int(rank if rank is not None else (tdist.get_rank(group) if ddp else 0))
        if minibatch <= 0 or minibatch % (64 * self.world):
            raise ValueError("minibatch must be a positive multiple of 64 x world")
        self.dp = self.world > 1 if data_parallel is None else bool(data_parallel)
        self.allreduce = allreduce or (lambda t: tdist.all_reduce(t, group=group))
        # torch.distributed's own all-reduce on an RCCL group can be captured into the epoch graph
        self.graph_collectives = allreduce is None and ddp and tdist.get_backend(group) == "nccl"
        dev = next(policy.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("FusedPPOTrainer runs on the GPU (HIP) only")
        self.policy, self.device = policy, dev
        self.global_minibatch = int(minibatch)
        self.minibatch = self.global_minibatch // self.world  # rows per rank and step
        offs, n = layout()
        params = list(policy.state_dict(keep_vars=True).values())
        if len(params) != len(offs):
            raise ValueError("unexpected state_dict layout")
        f32 = dict(dtype=torch.float32, device=dev)
        self.params = torch.zeros(n, **f32)
        with torch.no_grad():
            for p, o in zip(params, offs):
                self.params[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = self.params[o:o + p.numel()].view_as(p)
        self.grads = torch.zeros(n, **f32)
        self.adam_m = torch.zeros(n, **f32)
        self.adam_v = torch.zeros(n, **f32)
        self.adam_step = torch.zeros(1, dtype=torch.float64, device=dev)
        self.stats = torch.zeros(4, dtype=torch.float64, device=dev)
        self.loss_sums = torch.zeros(4, **f32)
        ws = LIB.uavhip_ppo_workspace_floats(self.minibatch)
        self.workspace = torch.zeros(int(ws), **f32)
        self.idx = torch.zeros(self.minibatch, dtype=torch.int32, device=dev)
        d = _lib.PPODesc()
        d.params, d.grads = self.params.data_ptr(), self.grads.data_ptr()
        d.adam_m, d.adam_v, d.adam_step = self.adam_m.data_ptr(), self.adam_v.data_ptr(), self.adam_step.data_ptr()
        d.workspace, d.stats, d.loss_sums = self.workspace.data_ptr(), self.stats.data_ptr(), self.loss_sums.data_ptr()
        d.n_floats, d.minibatch, d.global_minibatch = n, self.minibatch, self.global_minibatch
        d.lr_actor = cfg.LR_ACTOR if lr_actor is None else lr_actor
        d.lr_critic = cfg.LR_CRITIC if lr_critic is None else lr_critic
        d.beta1, d.beta2, d.adam_eps = betas[0], betas[1], adam_eps
        d.eps_clip = cfg.EPS_CLIP if eps_clip is None else eps_clip
        d.max_grad_norm = cfg.GRAD_NORM_CLIP if max_grad_norm is None else max_grad_norm
        d.value_coef, d.entropy_coef = value_coef, entropy_coef
        self.desc = d
        self.bufs = None
        self.graphs = {}    # steps per epoch -> captured epoch hipGraph over the current buffers
        self.capture_failed = {}  # steps per epoch -> why a (voted) capture failed: run() steps eagerly
        self._store = None  # stage(): the trainer's own trajectory buffers
        self._cap = 0
        self.n_local = None  # set_shard(): rows of this rank's shard

    def _restore_rows(self):
        """Back to minibatch / world rows per step after a set_shard() run resized the workspace to
        its padded owned-row count (gathered or single-GPU buffers slice minibatches by it)."""
        if self.minibatch != self.global_minibatch // self.world:
            self._resize(self.global_minibatch // self.world)

    def set_buffers(self, states, actions, old_logprobs, old_values, returns, advantages):
        """Trajectory buffers the minibatches are drawn from (kept by reference: a captured graph
        reads them at their current addresses)."""
        n = states.shape[0]
        dev = self.device
        self._restore_rows()
        self.bufs = (states.to(device=dev, dtype=torch.float32).contiguous().reshape(n, cfg.SEQ_LEN, cfg.STATE_DIM),
                     actions.to(device=dev, dtype=torch.int8).contiguous().reshape(n),
                     old_logprobs.to(device=dev, dtype=torch.float32).contiguous().reshape(n),
                     old_values.to(device=dev, dtype=torch.float32).contiguous().reshape(n),
                     returns.to(device=dev, dtype=torch.float32).contiguous().reshape(n),
                     advantages.to(device=dev, dtype=torch.float32).contiguous().reshape(n))
        self.n = n
        self.perm = torch.zeros(n, dtype=torch.int32, device=dev)  # the epoch's minibatch order
        self.graphs = {}
        self.capture_failed = {}
        self._store = None
        self.n_local = None

    def set_shard(self, states, actions, old_logprobs, old_values, returns, advantages):
        """Data parallel without a trajectory exchange: this rank's own rollout shard of n_local
        rows (the same count on every rank; global row g = rank * n_local + local row, the
        (rank, step, env) order RolloutEngine.gather() would produce). run() draws minibatches over
        the world * n_local global rows and each rank computes the ones it owns."""
        self.set_buffers(states, actions, old_logprobs, old_values, returns, advantages)
        self.n_local = self.n
        self.n = self.n_local * self.world

    def _resize(self, rows):
        """Rows per rank and step (a multiple of 64): workspace and row-index buffers for them."""
        ws = LIB.uavhip_ppo_workspace_floats(rows)
        self.workspace = torch.zeros(int(ws), dtype=torch.float32, device=self.device)
        self.idx = torch.zeros(rows, dtype=torch.int32, device=self.device)
        self.minibatch = rows
        self.desc.minibatch = rows
        self.desc.workspace = self.workspace.data_ptr()
        self.graphs = {}  # captured against the old workspace / row count

    def _owned(self, order, steps):
        """[steps, rows] this rank's rows of each global minibatch of `order` (global row indices,
        on the device), in minibatch order, padded with -1 to a common multiple of 64."""
        Bg = self.global_minibatch
        o = order[:steps * Bg].view(steps, Bg).long()
        mine = torch.div(o, self.n_local, rounding_mode="floor") == self.rank
        cnt = mine.sum(1)
        rows = max(64, -(-int(cnt.max().item()) // 64) * 64)  # one host sync per epoch
        first = torch.sort((~mine).to(torch.int8), dim=1, stable=True).indices[:, :rows]
        local = torch.gather(o, 1, first) - self.rank * self.n_local
        valid = torch.arange(rows, device=o.device)[None, :] < cnt[:, None]
        return torch.where(valid, local, torch.full_like(local, -1)).to(torch.int32), rows

    def stage(self, states, actions, old_logprobs, old_values, returns, advantages):
        """Copy a trajectory into the trainer's own device buffers (capacity grows in powers of two),
        so the epoch graphs captured for one size stay valid for the next update of any size they
        cover (PPOAgent.update: every update has a different buffer length)."""
        n = states.shape[0]
        dev = self.device
        self._restore_rows()
        if self._store is None or self._cap < n:
            cap = 1 << max(10, (n - 1).bit_length())
            f32 = dict(dtype=torch.float32, device=dev)
            self._store = (torch.zeros(cap, cfg.SEQ_LEN, cfg.STATE_DIM, **f32),
                           torch.zeros(cap, dtype=torch.int8, device=dev),
                           *(torch.zeros(cap, **f32) for _ in range(4)))
            self._cap = cap
            self.perm = torch.zeros(cap, dtype=torch.int32, device=dev)
            self.graphs = {}
        src = (states.reshape(n, cfg.SEQ_LEN, cfg.STATE_DIM), actions.reshape(n), old_logprobs.reshape(n),
               old_values.reshape(n), returns.reshape(n), advantages.reshape(n))
        for dst, x in zip(self._store, src):
            dst[:n].copy_(x)
        self.bufs = self._store
        self.n = n
        self.n_local = None

    def step(self, phases=_lib.PPO_FULL, idx=None):
        """uavhip_ppo_step phases (bit mask) on this rank's rows idx (default self.idx)."""
        s, a, lp, v, r, adv = self.bufs
        idx = self.idx if idx is None else idx
        check(LIB.uavhip_ppo_step(self.desc, ptr(s), ptr(a), ptr(lp), ptr(v), ptr(r), ptr(adv), ptr(idx),
                                  int(phases), stream_handle()), "uavhip_ppo_step")

    def _rows(self, perm, b):
        """This rank's rows of global minibatch b of the permutation perm (a view)."""
        Bg, Bl = self.global_minibatch, self.minibatch
        return perm[b * Bg + self.rank * Bl:b * Bg + (self.rank + 1) * Bl]

    @staticmethod
    def _packed(b):
        """Phase bit of minibatch step b of an epoch: every step after the first skips the repack
        of the weights (the previous step's UPDATE refreshed the packed copies, PPO_PACKED); the
        first repacks, so parameters changed between epochs (load_state_dict, ...) are picked up."""
        return _lib.PPO_PACKED if b > 0 else 0

    def ddp_step(self, idx=None, packed=0):
        """One data-parallel optimizer step (see the module docstring)."""
        self.step(_lib.PPO_FORWARD | packed, idx)
        self.allreduce(self.loss_sums)
        self.step(_lib.PPO_BACKWARD, idx)
        self.allreduce(self.grads)
        self.step(_lib.PPO_UPDATE, idx)

    def gradients(self, idx):
        """Raw gradients (before clipping) of the PPO loss on rows idx, as a flat tensor."""
        self.idx.copy_(torch.as_tensor(idx, dtype=torch.int32, device=self.device))
        self.step(_lib.PPO_FORWARD | _lib.PPO_BACKWARD)
        return self.grads

    #: an epoch of more minibatch steps than this is replayed as chunks of one captured graph of this
    #: many steps (each chunk's rows copied into the front of the permutation buffer first), so the
    #: reference's minibatch 64 over a whole rollout (4,096 steps per epoch at 4096 envs x 64) needs
    #: no 37 k-node graph
    max_graph_steps = 256

    def capture(self):
        """Capture one epoch (every minibatch step of the current buffer length, or a chunk of
        max_graph_steps of them) into a hipGraph; a data-parallel epoch with its RCCL all-reduces
        (every rank captures the same sequence, so the replays meet in the same collectives).
        Data parallel: the ranks vote on the capture (an all-reduce of a success flag after it); if
        any rank failed, every rank drops its graph and returns None, and run() steps eagerly on all
        of them -- no rank can go on into replays the others never join."""
        if self.dp and not self.graph_collectives:
            raise RuntimeError("graph capture of the data-parallel step needs torch.distributed's all-reduce on "
                               "an RCCL ('nccl') group; gloo collectives run eagerly")
        if self.dp and self.n_local is not None:
            raise RuntimeError("set_shard() epochs resize per epoch: they run eagerly")
        steps = min(self.n // self.global_minibatch, self.max_graph_steps)
        if self.dp:  # the communicator is created at its first collective, which must not be in a capture
            self.allreduce(torch.zeros(1, dtype=torch.float32, device=self.device))
            if self.device.type == "cuda":
                torch.cuda.synchronize()
        g, err = None, None
        try:
            g = self._capture_graph(steps)
        except Exception as exc:  # noqa: BLE001 -- data parallel: voted on below, then re-raised / eager
            g, err = None, exc
        if self.dp:
            ok = torch.tensor([0.0 if g is None else 1.0], dtype=torch.float32, device=self.device)
            self.allreduce(ok)
            if int(ok.item()) != self.world:
                # remembered per step count: later run()s step eagerly without voting again
                why = repr(err) if err is not None else f"the capture failed on {self.world - int(ok.item())} other rank(s)"
                self.capture_failed[steps] = why
                self.graphs.pop(steps, None)
                import sys
                print(f"[FusedPPOTrainer rank {self.rank}] epoch graph capture ({steps} steps) failed, "
                      f"eager steps: {why}", file=sys.stderr)
                return None
        elif err is not None:
            raise err
        self.graphs[steps] = g
        return g

    def _capture_graph(self, steps):
        """The capture itself: `steps` minibatch steps over perm into a new hipGraph."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        # thread_local: the process group's watchdog thread keeps polling its events during the capture
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local" if self.dp else "global"):
            for b in range(steps):  # one epoch (or chunk): every minibatch step
                if self.dp:
                    self.ddp_step(self._rows(self.perm, b), self._packed(b))
                else:
                    self.step(_lib.PPO_FULL | self._packed(b), self._rows(self.perm, b))
        torch.cuda.current_stream().wait_stream(s)
        return g

    @property
    def graph(self):
        return self.graphs.get(min(self.n // self.global_minibatch, self.max_graph_steps))

    def run(self, epochs=None, generator=None, use_graph=True, perms=None):
        """K epochs of minibatch steps over the buffers -> (mean actor loss, critic loss, entropy, n_steps).
        Minibatch order: torch.randperm(n, generator) per epoch (SubsetRandomSampler's draw,
        ppo.py:115), or the given `perms` ([epochs][n] row orders, e.g. recorded from the reference).
        Epochs of more than max_graph_steps steps replay the chunk graph once per chunk (its rows
        copied device-to-device into the front of the permutation buffer before each replay) and step
        the remainder eagerly: the same steps in the same order as one epoch graph."""
        epochs = cfg.K_EPOCHS if epochs is None else epochs
        if perms is not None:
            perms = [torch.as_tensor(p, dtype=torch.int32) for p in perms]
            epochs = len(perms)
            if any(p.numel() != self.n for p in perms):
                raise ValueError(f"perms: every epoch's order must list the {self.n} rows")
        use_graph = use_graph and (not self.dp or self.graph_collectives)
        steps = self.n // self.global_minibatch
        if self.n_local is not None and self.dp:
            return self._run_shard(epochs, generator, perms, steps)
        graph = self.graph if use_graph else None
        chunk = min(steps, self.max_graph_steps)
        if use_graph and graph is None and steps > 0 and chunk not in self.capture_failed:
            graph = self.capture()
        Bg = self.global_minibatch
        order_dev = None
        if graph is not None and steps > chunk:
            order_dev = torch.empty(self.n, dtype=torch.int32, device=self.device)
        self.stats.zero_()
        cnt = 0
        for ep in range(epochs):
            order = perms[ep] if perms is not None else torch.randperm(self.n, generator=generator)
            if order_dev is None:
                self.perm[:self.n].copy_(order)
                if graph is not None:
                    graph.replay()
                    cnt += steps
                    continue
                for b in range(steps):
                    self._eager_step(self.perm, b)
                    cnt += 1
                continue
            order_dev.copy_(order)
            for c in range(steps // chunk):  # whole chunks: the chunk graph over perm[:chunk * Bg]
                self.perm[:chunk * Bg].copy_(order_dev[c * chunk * Bg:(c + 1) * chunk * Bg])
                graph.replay()
                cnt += chunk
            for b in range(steps - steps % chunk, steps):  # the ragged rest, eager
                self._eager_step(order_dev, b)
                cnt += 1
        self.policy._packed_key = None  # parameters changed under torch's version counters: repack
        if cnt == 0:
            return 0.0, 0.0, 0.0, 0
        st = self.stats.tolist()
        return st[0] / st[3], st[1] / st[3], st[2] / st[3], cnt

    def _eager_step(self, perm, b):
        """Minibatch step b of the order in perm, launched directly (the first step of an epoch
        repacks; later ones reuse the copies the previous UPDATE refreshed)."""
        if not self.dp:
            self.step(_lib.PPO_FULL | self._packed(b), self._rows(perm, b))
        else:
            self.ddp_step(self._rows(perm, b), self._packed(b))

    def _run_shard(self, epochs, generator, perms, steps):
        """run() over a set_shard() batch: per epoch the global order (the same on every rank), this
        rank's owned rows of each global minibatch, then the data-parallel steps."""
        self.stats.zero_()
        cnt = 0
        for ep in range(epochs):
            order = perms[ep] if perms is not None else torch.randperm(self.n, generator=generator)
            rows, r = self._owned(order.to(self.device), steps)
            if r != self.minibatch:
                self._resize(r)
            for b in range(steps):
                self.ddp_step(rows[b], self._packed(b))
                cnt += 1
        self.policy._packed_key = None
        if cnt == 0:
            return 0.0, 0.0, 0.0, 0
        st = self.stats.tolist()
        return st[0] / st[3], st[1] / st[3], st[2] / st[3], cnt
