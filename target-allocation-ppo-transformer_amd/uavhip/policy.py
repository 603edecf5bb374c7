"""TransformerActorCritic with the reference's parameter names, shapes and initialisation
(networks/transformer_net.py:9-144), so its state_dict round-trips with the reference's
checkpoints (main_train.py:211,232) and `torch.manual_seed(s); TransformerActorCritic()` yields the
reference's initial weights.

Two execution paths:
  * `get_action` (rollout, no grad): the fused HIP forward of libuavhip.so (policy.hip) on packed
    weights -- every encoder GEMM as fp32-accurate split products on the f16 MFMA (two fp16 planes per
    operand, DESIGN.md 4a: 2^-22 relative per product for |x| in [2^-14, 65536); a larger operand
    makes its plane NaN and the outputs that read it non-finite), the embeddings and heads on the f32 MFMA; the action is drawn on device from Philox. GPU only: raises otherwise.
  * `evaluate` (PPO update, autograd): the module's own torch forward, used by the update (SURVEY 8f
    "next" row); also the torch fp32 reference the fused kernel is tested against.
"""
import ctypes
import itertools

import numpy as np
import torch
import torch.nn as nn
from torch.distributions import Categorical

from . import _lib
from ._lib import LIB, check, ptr, stream_handle
from .config import cfg
from .vec_env import check_out


def _ortho(layer, std=float(np.sqrt(2)), bias=0.0):
    """transformer_net.py:9-12: orthogonal weight (gain std), constant bias."""
    nn.init.orthogonal_(layer.weight, std)
    nn.init.constant_(layer.bias, bias)
    return layer


class _Trunk(nn.Module):
    """Linear(14->128)+ReLU embedding, learned position embedding, post-LN encoder stack
    (transformer_net.py:15-64). Attribute names fix the state_dict keys."""

    def __init__(self, num_layers):
        super().__init__()
        self.embedding = nn.Sequential(_ortho(nn.Linear(cfg.STATE_DIM, cfg.EMBED_DIM)), nn.ReLU())
        self.pos_embedding = nn.Parameter(torch.randn(1, cfg.SEQ_LEN, cfg.EMBED_DIM) * 0.02)
        layer = nn.TransformerEncoderLayer(d_model=cfg.EMBED_DIM, nhead=cfg.NUM_HEADS, dim_feedforward=256,
                                           dropout=0.0, batch_first=True)
        # nn.TransformerEncoder deep-copies `layer`: every layer starts from identical weights,
        # as in the reference.
        self.transformer = nn.TransformerEncoder(layer, num_layers=num_layers, enable_nested_tensor=False)

    def forward(self, x):
        pad = x.abs().sum(dim=-1) == 0          # all-zero window rows are padding ...
        pad[:, -1] = False                       # ... except the current step (transformer_net.py:52-54)
        h = self.embedding(x) + self.pos_embedding[:, :x.size(1), :]
        return self.transformer(h, src_key_padding_mask=pad)


_INSTANCES = itertools.count()


def _instance_seed():
    """splitmix64 of (torch.initial_seed(), instance number) -> 62-bit Philox key."""
    z = (torch.initial_seed() + 0x9E3779B97F4A7C15 * (1 + next(_INSTANCES))) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return (z ^ (z >> 31)) & (2 ** 62 - 1)


class TransformerActorCritic(nn.Module):
    def __init__(self):
        super().__init__()
        self.hidden_dim = cfg.EMBED_DIM
        self.actor_net = _Trunk(num_layers=1)
        self.actor_head = nn.Sequential(_ortho(nn.Linear(self.hidden_dim, 64)), nn.ReLU(),
                                        _ortho(nn.Linear(64, cfg.ACTION_DIM), std=0.01))
        self.critic_net = _Trunk(num_layers=2)
        self.critic_head = nn.Sequential(_ortho(nn.Linear(self.hidden_dim, 64)), nn.ReLU(),
                                         _ortho(nn.Linear(64, 1), std=1.0))
        self._packed = None
        self._packed_key = None
        self._desc = None
        # Philox key of the on-device action sampling: torch.initial_seed() (so torch.manual_seed
        # controls it, as it controls the reference's Categorical sampling, transformer_net.py:120)
        # mixed with a per-process instance count (separate instances sample independently). Nothing
        # is drawn from the CPU generator: the sampler permutations after construction (ppo.py:115)
        # stay the reference's. The counter starts at 0 per instance.
        self.sample_seed = _instance_seed()
        self._sample_offset = 0

    def forward(self, state):
        raise NotImplementedError("Please use get_action or evaluate.")

    def __getstate__(self):
        # the packed-weight cache and its ctypes descriptor are per-instance device state
        state = self.__dict__.copy()
        state["_packed"] = state["_packed_key"] = state["_desc"] = None
        return state

    # ------------------------------------------------------------------ torch path
    def heads(self, state):
        """-> logits [B, 2], value [B, 1] via the torch modules (autograd-capable)."""
        if state.dim() == 2:
            state = state.unsqueeze(0)
        logits = self.actor_head(self.actor_net(state)[:, -1, :])
        value = self.critic_head(self.critic_net(state)[:, -1, :])
        return logits, value

    def evaluate(self, state, action, validate=True):
        """transformer_net.py:124-144 -> (log_prob(action), value [B, 1], entropy).
        validate=False skips Categorical's argument check (a host sync; graph capture)."""
        logits, value = self.heads(state)
        dist = Categorical(torch.softmax(logits, dim=-1), validate_args=None if validate else False)
        return dist.log_prob(action), value, dist.entropy()

    # ------------------------------------------------------------------ fused HIP path
    def packed_weights(self):
        """Packed fp32 weight buffer in the layout of uavhip_policy_layout (repacked when any
        parameter changed: optimizer steps and load_state_dict bump tensor versions)."""
        params = list(self.state_dict(keep_vars=True).values())
        dev = params[0].device
        key = (dev, tuple(p._version for p in params), tuple(p.data_ptr() for p in params))
        if self._packed is not None and self._packed_key == key:
            return self._packed
        if dev.type == "cuda":
            # on the device (uavhip_policy_pack: one launch from the flat parameter buffer, bitwise the
            # host pack_weights, test_device_pack_matches_host_pack), in place when the buffer exists:
            # a captured hipGraph keeps pointing at it
            _, total = split_layout()
            if self._packed is None or self._packed.device != dev or self._packed.numel() != total:
                self._packed = torch.empty(total, dtype=torch.float32, device=dev)
            flat = _flat_parameters(params)
            check(LIB.uavhip_policy_pack(ptr(flat), ptr(self._packed), stream_handle()), "uavhip_policy_pack")
        else:
            self._packed = pack_weights(self.state_dict(), device=dev)
        self._packed_key = key
        d = _lib.PolicyDesc()
        d.weights = self._packed.data_ptr()
        d.n_floats = self._packed.numel()
        d.d_model, d.n_heads, d.d_ff, d.d_head_hidden = cfg.EMBED_DIM, cfg.NUM_HEADS, 256, 64
        d.actor_layers, d.critic_layers = 1, 2
        self._desc = d
        return self._packed

    def fused_forward(self, states, actions=None, action_out=None, logp=None, value=None, entropy=None,
                      logits=None, seed=None, offset=None, offset_dev=None, check_weights=True, rowproj=None,
                      step=0, fill=True):
        """Raw fused forward on [B, 5, 14] fp32 device windows; returns the output tensors.
        offset_dev: optional device uint64 [1] added to the sampling counter (graph replays);
        check_weights=False skips the repack check (caller guarantees the pack is current).
        rowproj (a rowproj_buffer(B) tensor) selects the window-sequence fast path
        (uavhip_policy_forward_rows): step = index of `states` in the sequence, fill = rebuild the
        cached rows (first call, new weights, or windows not advanced by one row)."""
        if states.device.type != "cuda":
            raise RuntimeError("the fused policy forward runs on the GPU (HIP) only")
        states = states.contiguous()
        if states.dtype != torch.float32:
            states = states.float()
        B = states.shape[0]
        if states.numel() != B * cfg.SEQ_LEN * cfg.STATE_DIM:
            raise ValueError(f"states must be [B, {cfg.SEQ_LEN}, {cfg.STATE_DIM}] (got {tuple(states.shape)})")
        if check_weights or self._packed is None:
            self.packed_weights()
        dev = states.device
        action_out = torch.empty(B, dtype=torch.int8, device=dev) if action_out is None else action_out
        logp = torch.empty(B, dtype=torch.float32, device=dev) if logp is None else logp
        value = torch.empty(B, dtype=torch.float32, device=dev) if value is None else value
        if actions is not None:
            actions = actions.to(device=dev, dtype=torch.int8).contiguous()
            check_out(actions, "actions", torch.int8, (B,), dev)
        for t, name, dt, tail in ((action_out, "action_out", torch.int8, ()), (logp, "logp", torch.float32, ()),
                                  (value, "value", torch.float32, ()), (entropy, "entropy", torch.float32, ()),
                                  (logits, "logits", torch.float32, (2,))):
            check_out(t, name, dt, (B,), dev, tail)
        if offset is None:
            offset = self._sample_offset
            self._sample_offset += B
        seed = self.sample_seed if seed is None else seed
        if rowproj is not None:
            if rowproj.numel() < LIB.uavhip_policy_rowproj_floats(B) or rowproj.dtype != torch.float32:
                raise ValueError("rowproj: need a float32 buffer of rowproj_buffer(B) elements")
            check(LIB.uavhip_policy_forward_rows(self._desc, ptr(states), B, ptr(rowproj), int(step), int(bool(fill)),
                                                 ptr(actions), ctypes.c_uint64(seed), ctypes.c_uint64(offset),
                                                 ptr(offset_dev), ptr(action_out), ptr(logp), ptr(value),
                                                 ptr(entropy), ptr(logits), stream_handle()),
                  "uavhip_policy_forward_rows")
            return action_out, logp, value, entropy, logits
        check(LIB.uavhip_policy_forward(self._desc, ptr(states), B, ptr(actions), ctypes.c_uint64(seed),
                                        ctypes.c_uint64(offset), ptr(offset_dev), ptr(action_out), ptr(logp), ptr(value),
                                        ptr(entropy), ptr(logits), stream_handle()), "uavhip_policy_forward")
        return action_out, logp, value, entropy, logits

    def value_rows(self, states, rowproj, step, value, fill=False):
        """uavhip_policy_value_rows: the critic's value of [B, 5, 14] fp32 device windows on the
        window-sequence ring (the rollout's bootstrap V(s_T)) -- fused_forward(rowproj=...)'s value,
        bitwise, without the actor trunk and sampling. The actor's ring row of this step is not
        written, so the next call on the sequence must fill (RolloutEngine refills every iteration).
        The weights must be packed (packed_weights())."""
        if self._packed is None:
            self.packed_weights()
        B = states.shape[0]
        check_out(states, "states", torch.float32, (B,), states.device, (cfg.SEQ_LEN, cfg.STATE_DIM))
        check_out(value, "value", torch.float32, (B,), states.device)
        if rowproj.numel() < LIB.uavhip_policy_rowproj_floats(B) or rowproj.dtype != torch.float32:
            raise ValueError("rowproj: need a float32 buffer of rowproj_buffer(B) elements")
        check(LIB.uavhip_policy_value_rows(self._desc, ptr(states), B, ptr(rowproj), int(step), int(bool(fill)),
                                           ptr(value), stream_handle()), "uavhip_policy_value_rows")
        return value

    def rollout_step(self, env, states, rowproj, step, fill, action_out, logp, value, obs_out, reward_out, done_out,
                     info_out=None, auto_reset=True, seed=None, offset=0, offset_dev=None):
        """uavhip_rollout_step: the window-row forward + sampling over env's E windows `states`
        and the env step of the sampled actions in one launch (VecUAVEnv `env`, N, M <= 64).
        The weights must be packed (packed_weights())."""
        if self._packed is None:
            self.packed_weights()
        E, dev = env.E, env.device
        env._check_obs(obs_out)
        check_out(states, "states", torch.float32, (E,), dev, (cfg.SEQ_LEN, cfg.STATE_DIM))
        if rowproj.numel() < LIB.uavhip_policy_rowproj_floats(E) or rowproj.dtype != torch.float32 or \
                not rowproj.is_contiguous():
            raise ValueError("rowproj: need a contiguous float32 rowproj_buffer(E)")
        for t, name, dt, tail in ((action_out, "action_out", torch.int8, ()), (logp, "logp", torch.float32, ()),
                                  (value, "value", torch.float32, ()), (reward_out, "reward_out", torch.float64, ()),
                                  (done_out, "done_out", torch.uint8, ()),
                                  (info_out, "info_out", torch.float64, (_lib.INFO_COUNT,))):
            check_out(t, name, dt, (E,), dev, tail)
        seed = self.sample_seed if seed is None else seed
        check(LIB.uavhip_rollout_step(self._desc, env.desc, ptr(states), ptr(rowproj), int(step), int(bool(fill)),
                                      ctypes.c_uint64(seed), ctypes.c_uint64(offset), ptr(offset_dev),
                                      ptr(action_out), ptr(logp), ptr(value), int(bool(auto_reset)), ptr(obs_out),
                                      ptr(reward_out), ptr(done_out), ptr(info_out), stream_handle()),
              "uavhip_rollout_step")

    def rollout_steps(self, env, obs, rowproj, step, fill, actions, logp, value, rewards, dones, info=None,
                      auto_reset=True, seed=None, offset=0, offset_stride=0, offset_dev=None):
        """uavhip_rollout_steps: n = actions.shape[0] consecutive rollout_step()s in one launch.
        obs [n + 1][E][5][14] f32 (obs[0] = the current windows; obs[t + 1] receives step t's next
        windows), actions / logp / value / rewards / dones [n][E], info [n][E][INFO_COUNT] or None;
        step t samples with counters offset + t * offset_stride + b (+ *offset_dev)."""
        if self._packed is None:
            self.packed_weights()
        E, dev = env.E, env.device
        n = actions.shape[0] if actions.dim() == 2 else -1
        if n <= 0:
            raise ValueError("actions: need an int8 [n][E] buffer with n > 0")
        check_out(obs, "obs", torch.float32, (n + 1, E), dev, (cfg.SEQ_LEN, cfg.STATE_DIM))
        if rowproj.numel() < LIB.uavhip_policy_rowproj_floats(E) or rowproj.dtype != torch.float32 or \
                not rowproj.is_contiguous():
            raise ValueError("rowproj: need a contiguous float32 rowproj_buffer(E)")
        for t, name, dt, tail in ((actions, "actions", torch.int8, ()), (logp, "logp", torch.float32, ()),
                                  (value, "value", torch.float32, ()), (rewards, "rewards", torch.float64, ()),
                                  (dones, "dones", torch.uint8, ()),
                                  (info, "info", torch.float64, (_lib.INFO_COUNT,))):
            check_out(t, name, dt, (n, E), dev, tail)
        seed = self.sample_seed if seed is None else seed
        check(LIB.uavhip_rollout_steps(self._desc, env.desc, ptr(obs), ptr(rowproj), int(step), int(n),
                                       int(bool(fill)), ctypes.c_uint64(seed), ctypes.c_uint64(offset),
                                       ctypes.c_uint64(offset_stride), ptr(offset_dev), ptr(actions), ptr(logp),
                                       ptr(value), int(bool(auto_reset)), ptr(rewards), ptr(dones), ptr(info),
                                       stream_handle()), "uavhip_rollout_steps")

    @torch.no_grad()
    def get_action(self, state):
        """transformer_net.py:96-122 -> (action [B] int64, log_prob [B], value [B, 1], entropy [B])."""
        if state.dim() == 2:
            state = state.unsqueeze(0)
        B = state.shape[0]
        ent = torch.empty(B, dtype=torch.float32, device=state.device)
        a, lp, v, ent, _ = self.fused_forward(state, entropy=ent)
        return a.long(), lp, v.view(B, 1), ent


def rowproj_buffer(B, device="cuda"):
    """Zeroed window-row projection buffer for fused_forward(rowproj=...) over B windows."""
    return torch.zeros(int(LIB.uavhip_policy_rowproj_floats(int(B))), dtype=torch.float32, device=device)


def layout():
    n = LIB.uavhip_policy_layout(None, 0)
    offs = (ctypes.c_int32 * 64)()
    LIB.uavhip_policy_layout(offs, 64)
    return [offs[i] for i in range(50)], int(n)


def tiling():
    """In-features K of each parameter stored in MFMA fragment order (0 = flat), key order."""
    kc = (ctypes.c_int32 * 64)()
    np_ = LIB.uavhip_policy_tiling(kc, 64)
    return [kc[i] for i in range(np_)]


def split_layout():
    """[(state_dict index, float offset)] of the split weight copies and the packed buffer's total
    floats (include/uavhip.h uavhip_policy_split_layout)."""
    params, offs = (ctypes.c_int32 * 16)(*([-1] * 16)), (ctypes.c_int32 * 16)()
    total = LIB.uavhip_policy_split_layout(params, offs, 16)
    return [(params[i], offs[i]) for i in range(16) if params[i] >= 0], int(total)


def to_split_fragment_order(w):
    """[R][K] fp32 -> the split copy as float32 words: two fp16 planes w1 = f16(w),
    w2 = f16((w - w1) * 2^11) in blocks of 16 rows x 32 k (1 KiB of w1, then 1 KiB of w2), lane
    l = r%16 + 16 ((k%32)//8) holding k%8 = 0..7 (the f16 MFMA operand layout, policy.hip hgemm_tile)."""
    R, K = w.shape
    w = w.to(torch.float32)
    w1 = w.to(torch.float16)  # IEEE round-to-nearest, inf beyond 65504: what the device conversions do
    w2 = ((w - w1.to(torch.float32)) * 2048.0).to(torch.float16)

    def frag(p):
        return p.reshape(R // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(R // 16, K // 32, 512)

    return torch.stack([frag(w1), frag(w2)], dim=2).reshape(-1).view(torch.float32)


def to_fragment_order(w, K):
    """[R][K] -> MFMA fragment order (include/uavhip.h uavhip_policy_tiling): blocks of 16 rows x
    16 k, inside a block lane = r%16 + 16 * ((k%16)//4) holds k%4 = 0..3."""
    R = w.shape[0]
    return w.reshape(R // 16, 16, K // 16, 4, 4).permute(0, 2, 3, 1, 4).reshape(-1)


def from_fragment_order(flat, R, K):
    return flat.reshape(R // 16, K // 16, 4, 16, 4).permute(0, 3, 1, 2, 4).reshape(R, K)


def _flat_parameters(params):
    """The parameters as one flat fp32 device buffer in the uavhip_policy_layout() order: the storage
    itself when every parameter is already a view at its layout offset of one buffer
    (FusedPPOTrainer's), else a copy (padding floats zero)."""
    offs, n = layout()
    p0 = params[0]
    st = p0.untyped_storage()
    base = st.data_ptr()
    if all(p.dtype == torch.float32 and p.is_contiguous() and p.untyped_storage().data_ptr() == base for p in params):
        start = p0.data_ptr() - 4 * offs[0]
        if (start - base) % 4 == 0 and start >= base and start - base + 4 * n <= st.nbytes() and \
                all(p.data_ptr() == start + 4 * o for p, o in zip(params, offs)):
            return torch.empty(0, dtype=torch.float32, device=p0.device).set_(st, (start - base) // 4, (n,))
    flat = torch.zeros(n, dtype=torch.float32, device=p0.device)
    for p, o in zip(params, offs):
        flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
    return flat


def pack_weights(state_dict, device=None):
    """Lay the 50-key state_dict out as the kernel's packed buffer (state_dict key order; GEMM
    weights in MFMA fragment order), followed by the split copies (split_layout())."""
    offs, n = layout()
    kcols = tiling()
    items = list(state_dict.items())
    if len(items) != len(offs) or len(kcols) != len(offs):
        raise ValueError(f"expected {len(offs)} state_dict entries, got {len(items)}")
    dev = device if device is not None else items[0][1].device
    splits, total = split_layout()
    buf = torch.zeros(total, dtype=torch.float32, device=dev)
    ends = offs[1:] + [n]
    for (k, v), o, e, K in zip(items, offs, ends, kcols):
        v = v.detach().to(device=dev, dtype=torch.float32)
        if K:
            if v.dim() != 2 or v.shape[1] != K or v.shape[0] % 16:
                raise ValueError(f"{k}: shape {tuple(v.shape)} is not [16 r][{K}]")
            flat = to_fragment_order(v, K)
        else:
            flat = v.reshape(-1)
        if flat.numel() > e - o:
            raise ValueError(f"{k}: {flat.numel()} floats do not fit the packed slot {e - o}")
        buf[o:o + flat.numel()] = flat
    for q, o in splits:  # the split copies of the f16-matrix-core GEMM weights
        flat = to_split_fragment_order(items[q][1].detach().to(device=dev, dtype=torch.float32))
        buf[o:o + flat.numel()] = flat
    if RANGE_FLOATS:  # the packed table holds the maxima only (the kernels derive the scales)
        t = range_table([v for _, v in items])
        t[len(items):] = 0.0
        buf[total - RANGE_FLOATS:] = t.to(dev)
    return buf


# (0 only for an A/B timing build of the previous ABI, which has no range table: _lib)
RANGE_FLOATS = int(LIB.uavhip_policy_range_table(None, None)) if hasattr(LIB, "uavhip_policy_range_table") else 0


def range_table(params):
    """The range table (include/uavhip.h uavhip_policy_range_table) of the 50 parameters: their max
    |value|, then the scales of the split products' operands derived from them by the library's own
    host code -- bitwise what every kernel derives from the maxima, the part of the table the packed
    buffer carries (pack_weights)."""
    # NaN elements are ignored, as the device's reductions do (k_policy_range / k_adam reduce with
    # fmaxf, which drops NaN): the host and device tables agree bitwise for any parameter
    m = torch.tensor([float(torch.nan_to_num(p.detach().abs().float(), nan=0.0, posinf=float("inf")).max())
                      for p in params], dtype=torch.float32)
    out = torch.zeros(RANGE_FLOATS, dtype=torch.float32)
    LIB.uavhip_policy_range_table(ctypes.c_void_p(m.data_ptr()), ctypes.c_void_p(out.data_ptr()))
    return out
