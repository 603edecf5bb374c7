"""VecUAVEnv: E independent UAVEnv instances (envs/uav_env.py:13) resident in HBM as SoA tensors,
stepped by the HIP kernels of libuavhip.so (include/uavhip.h).

This is the batched fast path. The reference steps one Python object per call
(`UAVEnv.step`, uav_env.py:295-435); here one launch steps all E envs (and optionally T
consecutive steps). `envs/uav_env.py` in this package is the E = 1 drop-in view.
"""
import numpy as np
import torch

from . import _lib
from ._lib import LIB, check, ptr, stream_handle
from .config import cfg as default_cfg, gen_vector, params_vector

SCENE_KEYS_F64 = ("uav_pos", "uav_vel", "uav_load", "uav_cost", "tgt_pos", "tgt_vel", "tgt_value", "nfz_pos",
                  "icp_pos", "icp_vel")


def _same_device(t, device):
    return t.device.type == device.type and (device.index is None or t.device.index == device.index)


def check_out(t, name, dtype, lead, device, tail=()):
    """A caller-provided kernel buffer (read or written through a raw pointer): right device and
    dtype, contiguous, exactly prod(lead + tail) elements -- anything else would be an out-of-bounds
    or misread device access the C side cannot detect. None passes (NULL = not wanted)."""
    if t is None:
        return
    n = 1
    for d in tuple(lead) + tuple(tail):
        n *= int(d)
    if not isinstance(t, torch.Tensor) or not _same_device(t, device) or t.dtype != dtype or \
            not t.is_contiguous() or t.numel() != n:
        got = (f"{t.dtype} {tuple(t.shape)} on {t.device}, contiguous={t.is_contiguous()}"
               if isinstance(t, torch.Tensor) else type(t).__name__)
        raise ValueError(f"{name}: need a contiguous {dtype} tensor of {n} elements on {device} (got {got})")


class VecUAVEnv:
    def __init__(self, num_envs, num_uavs=None, num_targets=None, num_nfz=None, num_interceptors=None, config=None,
                 device="cuda", seed=0, full_reset_period=None, scene_buffers=None, obs_dtype=torch.float32,
                 env_base=0):
        """obs_dtype: float32, or float16 (BASELINE config 4: observations emitted as IEEE binary16,
        UAVHIP_ENV_OBS_F16; the env's own window deque stays f32).
        env_base: global index of env 0 when this is one rank's shard of a larger env set -- the
        on-device scenes of env e are those of env env_base + e of the union (uavhip_env.env_base)."""
        c = config or default_cfg
        if obs_dtype not in (torch.float32, torch.float16):
            raise ValueError(f"obs_dtype must be torch.float32 or torch.float16 (got {obs_dtype})")
        self.obs_dtype = obs_dtype
        self.cfg = c
        self.E = int(num_envs)
        self.N = int(num_uavs if num_uavs is not None else c.NUM_UAVS)
        self.M = int(num_targets if num_targets is not None else c.NUM_TARGETS)
        self.Kn = int(num_nfz if num_nfz is not None else c.NUM_NFZ)
        self.Ki = int(num_interceptors if num_interceptors is not None else c.NUM_INTERCEPTORS)
        if not (1 <= self.N <= _lib.MAX_N and 1 <= self.M <= _lib.MAX_M):
            raise ValueError(f"N={self.N} (<= {_lib.MAX_N}) / M={self.M} (<= {_lib.MAX_M}) out of range")
        if not (0 <= self.Kn <= _lib.MAX_OBSTACLES and 0 <= self.Ki <= _lib.MAX_OBSTACLES):
            raise ValueError("too many obstacles")
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("VecUAVEnv runs on the GPU (HIP) only; the CPU oracle lives in oracle/ (tests)")
        period = c.FULL_RESET_PERIOD if full_reset_period is None else int(full_reset_period)
        B = (2 if period > 0 else 1) if scene_buffers is None else int(scene_buffers)
        self.period, self.B = period, B
        E, N, M, Kn, Ki = self.E, self.N, self.M, self.Kn, self.Ki
        f64 = dict(dtype=torch.float64, device=self.device)
        i32 = dict(dtype=torch.int32, device=self.device)
        z = torch.zeros
        # scene arrays and pair tables: [B * E, ...]; env e's active scene is row sel * E + e
        self._scene = dict(
            uav_pos=z(B * E, N, 2, **f64), uav_vel=z(B * E, N, 2, **f64), uav_load=z(B * E, N, **f64),
            uav_cost=z(B * E, N, **f64), uav_type=z(B * E, N, **i32), tgt_pos=z(B * E, M, 2, **f64),
            tgt_vel=z(B * E, M, 2, **f64), tgt_value=z(B * E, M, **f64), tgt_id=z(B * E, M, **i32),
            nfz_pos=z(B * E, max(Kn, 1), 2, **f64), icp_pos=z(B * E, max(Ki, 1), 2, **f64),
            icp_vel=z(B * E, max(Ki, 1), 2, **f64), p_dmg=z(B * E, N, M, **f64), p_pen=z(B * E, N, **f64))
        self.nh_final, self.nh_pure = z(E, M, **f64), z(E, M, **f64)
        self.t_cost, self.n_lock = z(E, M, **f64), z(E, M, **i32)
        self.assigned = torch.full((E, N), -1, **i32)
        self.istate = z(E, _lib.IST_COUNT, **i32)
        self.dstate = z(E, _lib.DST_COUNT, **f64)
        self.window = z(E, _lib.SEQ_LEN, _lib.STATE_DIM, dtype=torch.float32, device=self.device)
        d = _lib.EnvDesc()
        d.E, d.N, d.M, d.Kn, d.Ki = E, N, M, Kn, Ki
        d.full_reset_period = period
        d.scene_buffers = B
        d.seed = int(seed) & (2 ** 64 - 1)
        self.env_base = int(env_base)
        if self.env_base < 0:
            raise ValueError("env_base must be >= 0")
        d.env_base = self.env_base
        d.flags = _lib.ENV_OBS_F16 if obs_dtype == torch.float16 else 0
        for i, v in enumerate(params_vector(c)):
            d.prm[i] = float(v)
        for i, v in enumerate(gen_vector(c)):
            d.gen[i] = float(v)
        for name, t in self._scene.items():
            setattr(d, name, t.data_ptr())
        for name in ("nh_final", "nh_pure", "t_cost", "n_lock", "assigned", "istate", "dstate", "window"):
            setattr(d, name, getattr(self, name).data_ptr())
        self.desc = d
        # per-step output buffers (reused; [E] views of the T=1 case)
        self._obs = torch.zeros(E, _lib.SEQ_LEN, _lib.STATE_DIM, dtype=obs_dtype, device=self.device)
        self._rew = torch.zeros(E, **f64)
        self._done = torch.zeros(E, dtype=torch.uint8, device=self.device)
        self._info = torch.zeros(E, _lib.INFO_COUNT, **f64)

    # ------------------------------------------------------------------ scenes
    def scene_sel(self):
        return (self.istate[:, _lib.IST["SCENE_SEL"]] & 1).long() if self.B == 2 else \
            torch.zeros(self.E, dtype=torch.long, device=self.device)

    def active(self, name):
        """Env-indexed [E, ...] copy of scene array `name` from each env's active buffer."""
        t = self._scene[name]
        if self.B == 1:
            return t
        rows = self.scene_sel() * self.E + torch.arange(self.E, device=self.device)
        return t[rows]

    def __getattr__(self, name):
        scene = self.__dict__.get("_scene")
        if scene is not None and name in scene:
            return self.active(name)
        raise AttributeError(name)

    def set_params(self, params):
        for i, v in enumerate(np.asarray(params, np.float64)):
            self.desc.prm[i] = float(v)

    def load_scenes(self, scenes, env_ids=None):
        """Copy host scenes (dicts in the tests/golden / scene.generate_scene layout) into buffer 0
        of envs `env_ids` (default 0..len-1), make it their active scene, rescore it. With two
        buffers the spare is marked stale (uavhip_scene_refresh fills it on device).
        A scene with a negative target value turns the omega = 0 replay kernel off for this env set
        (UAVHIP_ENV_NO_REPLAY: K2r needs every assign accepted, i.e. values >= 0)."""
        if isinstance(scenes, dict):
            scenes = [scenes]
        if any(np.size(s["tgt_value"]) and float(np.min(s["tgt_value"])) < 0 for s in scenes):
            self.desc.flags |= _lib.ENV_NO_REPLAY
        ids = list(range(len(scenes))) if env_ids is None else list(env_ids)
        mask = torch.zeros(self.E, dtype=torch.uint8)
        for e, s in zip(ids, scenes):
            for k in SCENE_KEYS_F64:
                dst = self._scene[k][e]
                src = torch.as_tensor(np.asarray(s[k], np.float64).reshape(dst.shape) if np.size(s[k]) else
                                      np.zeros(dst.shape))
                dst.copy_(src)
            self._scene["tgt_id"][e].copy_(torch.as_tensor(np.asarray(s["tgt_id"], np.int32)))
            if "uav_type" in s:
                self._scene["uav_type"][e].copy_(torch.as_tensor(np.asarray(s["uav_type"], np.int32)))
            self.istate[e, _lib.IST["SCENE_SEL"]] = 0
            self.istate[e, _lib.IST["SCENE_STALE"]] = 1 if self.B == 2 else 0
            mask[e] = 1
        self.score_pairs(mask.to(self.device))
        return mask

    def score_pairs(self, mask=None):
        check_out(mask, "mask", torch.uint8, (self.E,), self.device)
        check(LIB.uavhip_score_pairs(self.desc, ptr(mask), stream_handle()), "uavhip_score_pairs")

    def generate_scenes(self, mask=None):
        """On-device Philox scenes (distribution of uav_env.py:65-173) + pair tables, for the
        active buffer and (double-buffered) the spare."""
        check_out(mask, "mask", torch.uint8, (self.E,), self.device)
        check(LIB.uavhip_scene_generate(self.desc, ptr(mask), stream_handle()), "uavhip_scene_generate")

    def refresh_scenes(self):
        """Regenerate spares consumed by full resets (call once per rollout iteration)."""
        check(LIB.uavhip_scene_refresh(self.desc, stream_handle()), "uavhip_scene_refresh")

    # ------------------------------------------------------------------ reset / step
    def _check_obs(self, obs, lead=None):
        if obs is not None and obs.dtype != self.obs_dtype:
            raise TypeError(f"obs_out must be {self.obs_dtype} (got {obs.dtype})")
        check_out(obs, "obs_out", self.obs_dtype, (self.E,) if lead is None else lead, self.device,
                  (_lib.SEQ_LEN, _lib.STATE_DIM))

    def reset(self, mask=None, episode=-1, obs_out=None):
        self._check_obs(obs_out)
        check_out(mask, "mask", torch.uint8, (self.E,), self.device)
        out = self._obs if obs_out is None else obs_out
        check(LIB.uavhip_env_reset(self.desc, ptr(mask), int(episode), ptr(out), stream_handle()), "uavhip_env_reset")
        return out

    def step(self, actions, auto_reset=True, obs_out=None, reward_out=None, done_out=None, info_out=None,
             want_info=True):
        """actions: int8 tensor [E] (one step) or [T, E] (T fused steps). Returns (obs, reward,
        done, info) device tensors shaped [E, ...] or [T, E, ...]."""
        if actions.dtype != torch.int8 or actions.device != self.device:
            actions = actions.to(device=self.device, dtype=torch.int8)
        actions = actions.contiguous()
        T = 1 if actions.dim() == 1 else actions.shape[0]
        if actions.numel() != T * self.E:
            raise ValueError(f"actions must be [E]={self.E} or [T, E]")
        lead = (self.E,) if actions.dim() == 1 else (T, self.E)
        if T == 1 and actions.dim() == 1:
            obs = self._obs if obs_out is None else obs_out
            rew = self._rew if reward_out is None else reward_out
            done = self._done if done_out is None else done_out
            info = (self._info if info_out is None else info_out) if want_info else None
        else:
            dev = self.device
            obs = obs_out if obs_out is not None else torch.empty(*lead, _lib.SEQ_LEN, _lib.STATE_DIM,
                                                                  dtype=self.obs_dtype, device=dev)
            rew = reward_out if reward_out is not None else torch.empty(*lead, dtype=torch.float64, device=dev)
            done = done_out if done_out is not None else torch.empty(*lead, dtype=torch.uint8, device=dev)
            info = (info_out if info_out is not None else
                    torch.empty(*lead, _lib.INFO_COUNT, dtype=torch.float64, device=dev)) if want_info else None
        self._check_obs(obs, lead)
        check_out(rew, "reward_out", torch.float64, lead, self.device)
        check_out(done, "done_out", torch.uint8, lead, self.device)
        check_out(info, "info_out", torch.float64, lead, self.device, (_lib.INFO_COUNT,))
        check(LIB.uavhip_env_step(self.desc, ptr(actions), T, int(bool(auto_reset)), ptr(obs), ptr(rew), ptr(done),
                                  ptr(info), stream_handle()), "uavhip_env_step")
        return obs, rew, done, info

    # ------------------------------------------------------------------ state views
    def pointers(self):
        ist = self.istate[:, :2]
        return ist[:, 0], ist[:, 1]

    def assigned_target_ids(self):
        """UAV.assigned_target_id (entities.py:29) per env: the reference's target ids, -1 if none."""
        a = self.assigned.long()
        ids = torch.gather(self.tgt_id.long(), 1, a.clamp(min=0))
        return torch.where(a >= 0, ids, torch.full_like(ids, -1))

    def episodes(self):
        return self.istate[:, _lib.IST["EPISODE"]]

    def errors(self):
        return self.istate[:, _lib.IST["ERROR"]]
