"""Drop-in for the reference's envs/uav_env.py: `UAVEnv` with the same constructor, reset/step
signatures, return types and attributes (uav_env.py:13-435), as an E = 1 view over the HIP
VecUAVEnv. One step = one fused kernel launch + one 360-byte device->host copy.

Scenes come from uavhip.scene.generate_scene, which draws from the global numpy / `random`
streams in the reference's call order, so seeding as the reference is seeded reproduces its
scenes. `uavs`, `targets`, `nfz_list`, `interceptors` are entity views (envs/entities.py) built
on access from the device state.
"""
import numpy as np
import torch

from uavhip import _lib
from uavhip.config import cfg
from uavhip.scene import generate_scene
from uavhip.vec_env import VecUAVEnv

from envs.entities import UAV, Interceptor, NoFlyZone, Target


class _Discrete:
    def __init__(self, n):
        self.n = n


class _Box:
    def __init__(self, low, high, shape, dtype):
        self.low, self.high, self.shape, self.dtype = low, high, shape, dtype


# staging layout (bytes) of one step's outputs, copied to the host in one transfer
_OBS_B, _REW_B, _INFO_B, _DONE_B, _STAGE = 0, 280, 288, 352, 368


class UAVEnv:
    def __init__(self):
        self.action_space = _Discrete(cfg.ACTION_DIM)
        self.observation_space = _Box(-np.inf, np.inf, (cfg.SEQ_LEN, cfg.STATE_DIM), np.float32)
        self.uav_idx = 0
        self.target_idx = 0
        self.total_swarm_cost = 0.0
        self._venv = None
        self._scene = None
        self._done = True
        self._assigned_host = None

    # ------------------------------------------------------------------ internals
    def _ensure(self, N, M, Kn, Ki):
        v = self._venv
        if v is None or (v.N, v.M, v.Kn, v.Ki) != (N, M, Kn, Ki):
            self._venv = VecUAVEnv(1, N, M, Kn, Ki, config=cfg, full_reset_period=0)
            dev = self._venv.device
            self._act = torch.zeros(1, dtype=torch.int8, device=dev)
            self._stage = torch.zeros(_STAGE, dtype=torch.uint8, device=dev)
            self._obs_v = self._stage[_OBS_B:_REW_B].view(torch.float32).view(1, cfg.SEQ_LEN, cfg.STATE_DIM)
            self._rew_v = self._stage[_REW_B:_INFO_B].view(torch.float64)
            self._info_v = self._stage[_INFO_B:_DONE_B].view(torch.float64).view(1, _lib.INFO_COUNT)
            self._done_v = self._stage[_DONE_B:_DONE_B + 1]
        return self._venv

    def _generate_scene(self):
        s = generate_scene(cfg)
        self._scene = s
        self.total_swarm_cost = s["total_swarm_cost"]
        v = self._ensure(len(s["uav_load"]), len(s["tgt_value"]), len(s["nfz_pos"]), len(s["icp_pos"]))
        v.set_params(np.array([cfg.PARAM_ZETA_D, cfg.PARAM_K, cfg.PARAM_C1, cfg.PARAM_C2, cfg.PARAM_C3,
                               cfg.PARAM_C4, cfg.COST_WEIGHT_OMEGA, cfg.OBSTACLE_ZETA]))
        v.load_scenes(s)

    # ------------------------------------------------------------------ API (uav_env.py:42-63, 295-435)
    def reset(self, full_reset=True):
        if full_reset or self._venv is None:
            self._generate_scene()
        v = self._venv
        v.reset(episode=1, obs_out=self._obs_v)
        self._done = False
        self.uav_idx, self.target_idx = 0, 0
        self._assigned_host = None
        return self._obs_v[0].cpu().numpy().copy()

    def step(self, action):
        if self._done:
            raise IndexError("list index out of range")  # uav_env.py:296 on a finished episode
        self._act.fill_(int(action))
        self._venv.step(self._act, auto_reset=False, obs_out=self._obs_v, reward_out=self._rew_v,
                        done_out=self._done_v, info_out=self._info_v)
        host = self._stage.cpu().numpy()
        reward = float(host[_REW_B:_INFO_B].view(np.float64)[0])
        info_v = host[_INFO_B:_DONE_B].view(np.float64)
        done = bool(host[_DONE_B])
        self.uav_idx = int(info_v[_lib.INFO["UAV_IDX"]])
        self.target_idx = int(info_v[_lib.INFO["TARGET_IDX"]])
        self._done = done
        self._assigned_host = None
        obs = (np.zeros(cfg.STATE_DIM, dtype=np.float32) if done else
               host[_OBS_B:_REW_B].view(np.float32).reshape(cfg.SEQ_LEN, cfg.STATE_DIM).copy())
        iv = info_v[_lib.INFO["IS_VALID"]]
        info = {
            "J_val": float(info_v[_lib.INFO["J"]]),
            "num_assigned": int(info_v[_lib.INFO["NUM_ASSIGNED"]]),
            "is_valid_action": None if iv < 0 else bool(iv > 0),
            "avg_p_dmg": float(info_v[_lib.INFO["AVG_P_DMG"]]),
            "avg_p_final": float(info_v[_lib.INFO["AVG_P_FINAL"]]),
        }
        return obs, reward, done, info

    # ------------------------------------------------------------------ entity views
    def _assigned(self):
        if self._assigned_host is None:
            self._assigned_host = (self._venv.assigned[0].cpu().numpy(), self._venv.assigned_target_ids()[0].cpu().numpy())
        return self._assigned_host

    @property
    def uavs(self):
        s = self._scene
        if s is None:
            return []
        _, ids = self._assigned()
        out = []
        for i in range(len(s["uav_load"])):
            out.append(UAV(id=i, pos=s["uav_pos"][i].copy(), velocity=s["uav_vel"][i].copy(),
                           max_speed=float(s["uav_maxspeed"][i]), load=float(s["uav_load"][i]),
                           uav_type=int(s["uav_type"][i]), cost=float(s["uav_cost"][i]),
                           assigned_target_id=int(ids[i]), available=bool(ids[i] < 0)))
        return out

    @property
    def targets(self):
        s = self._scene
        if s is None:
            return []
        lidx, _ = self._assigned()
        out = []
        for t in range(len(s["tgt_value"])):
            out.append(Target(id=int(s["tgt_id"][t]), pos=s["tgt_pos"][t].copy(), value=float(s["tgt_value"][t]),
                              locked_by_uavs=[int(u) for u in np.nonzero(lidx == t)[0]],
                              velocity=s["tgt_vel"][t].copy()))
        return out

    @property
    def nfz_list(self):
        s = self._scene
        if s is None:
            return []
        return [NoFlyZone(id=i, pos=s["nfz_pos"][i].copy(), radius=float(s["nfz_radius"][i]))
                for i in range(len(s["nfz_pos"]))]

    @property
    def interceptors(self):
        s = self._scene
        if s is None:
            return []
        return [Interceptor(id=i, pos=s["icp_pos"][i].copy(), radius=float(s["icp_radius"][i]),
                            velocity=s["icp_vel"][i].copy()) for i in range(len(s["icp_pos"]))]
