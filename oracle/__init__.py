"""CPU ORACLE -- test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's ``cpu_baseline`` leg may import this
package, and only as the checker / the timed CPU baseline. The product package never
imports it (and fails loudly without its HIP library instead of falling back here).

Contents
  * ``uav_oracle.c`` (built to ``libuav_oracle.so`` by ``oracle/Makefile``): literal fp64
    restatement of envs/mechanics.py and UAVEnv.step/reset (reference recompute-from-scratch
    algorithm), wrapped here by :class:`OracleEnv` and :func:`score_pairs`.
  * :mod:`oracle.gae`: numpy fp32 restatement of agents/ppo.py:68-94 (GAE + adv. norm).
  * :mod:`oracle.policy_ref`: explicit torch-fp32 restatement of networks/transformer_net.py.

Pinned against tests/golden/*.npz, produced by running the reference itself
(tests/golden/make_golden.py; numpy 2.2.6 / torch 2.10 CPU).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

SEQ_LEN, STATE_DIM = 5, 14
INFO_FIELDS = ("J_val", "num_assigned", "is_valid", "avg_p_dmg", "avg_p_final", "uav_idx", "target_idx")

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)
_fp = ctypes.POINTER(ctypes.c_float)


def build():
    """Compile libuav_oracle.so in place (gcc)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libuav_oracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.uo_angle_score.restype = ctypes.c_double
        L.uo_angle_score.argtypes = [_dp, _dp, _dp]
        L.uo_speed_score.restype = ctypes.c_double
        L.uo_speed_score.argtypes = [ctypes.c_double, ctypes.c_double, _dp]
        L.uo_dist_score.restype = ctypes.c_double
        L.uo_dist_score.argtypes = [ctypes.c_double, ctypes.c_int, _dp]
        L.uo_damage_prob.restype = ctypes.c_double
        L.uo_damage_prob.argtypes = [_dp, _dp, ctypes.c_double, _dp, _dp, _dp]
        L.uo_penetration_prob.restype = ctypes.c_double
        L.uo_penetration_prob.argtypes = [_dp, _dp, _dp, ctypes.c_int, _dp, _dp, ctypes.c_int, _dp]
        L.uo_score_pairs.restype = None
        L.uo_score_pairs.argtypes = [ctypes.c_int] * 4 + [_dp] * 9 + [_dp, _dp]
        L.uo_env_create.restype = ctypes.c_void_p
        L.uo_env_create.argtypes = [ctypes.c_int] * 4 + [_dp] * 7 + [_ip] + [_dp] * 4
        L.uo_env_destroy.argtypes = [ctypes.c_void_p]
        L.uo_env_reset.argtypes = [ctypes.c_void_p, _fp]
        L.uo_env_step.restype = ctypes.c_int
        L.uo_env_step.argtypes = [ctypes.c_void_p, ctypes.c_int, _fp, _dp, _ip, _dp]
        L.uo_env_uav_idx.restype = ctypes.c_int
        L.uo_env_uav_idx.argtypes = [ctypes.c_void_p]
        L.uo_env_target_idx.restype = ctypes.c_int
        L.uo_env_target_idx.argtypes = [ctypes.c_void_p]
        L.uo_env_assigned.argtypes = [ctypes.c_void_p, _ip]
        L.uo_envs_run.restype = ctypes.c_long
        L.uo_envs_run.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.POINTER(ctypes.c_int8),
                                  ctypes.c_int, _fp]
        _LIB = L
    return _LIB


def _d(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(_dp)


def angle_score(up, uv, pt):
    (a, pa), (b, pb), (c, pc) = _d(up), _d(uv), _d(pt)
    return lib().uo_angle_score(pa, pb, pc)


def speed_score(us, ts, params):
    p, pp = _d(params)
    return lib().uo_speed_score(float(us), float(ts), pp)


def dist_score(d, obstacle, params):
    p, pp = _d(params)
    return lib().uo_dist_score(float(d), int(bool(obstacle)), pp)


def damage_prob(up, uv, load, tp, tv, params):
    args = [_d(x) for x in (up, uv, tp, tv, params)]
    return lib().uo_damage_prob(args[0][1], args[1][1], float(load), args[2][1], args[3][1], args[4][1])


def penetration_prob(up, uv, nfz_pos, icp_pos, icp_vel, params):
    nfz_pos = np.asarray(nfz_pos, np.float64).reshape(-1, 2)
    icp_pos = np.asarray(icp_pos, np.float64).reshape(-1, 2)
    icp_vel = np.asarray(icp_vel, np.float64).reshape(-1, 2)
    a = [_d(x) for x in (up, uv, nfz_pos, icp_pos, icp_vel, params)]
    return lib().uo_penetration_prob(a[0][1], a[1][1], a[2][1], len(nfz_pos), a[3][1], a[4][1], len(icp_pos),
                                     a[5][1])


def score_pairs(scene, params):
    """Dense (p_dmg[N,M], p_pen[N]) for one scene dict (tests/golden layout)."""
    N = len(scene["uav_load"]); M = len(scene["tgt_value"])
    nfz = np.asarray(scene["nfz_pos"], np.float64).reshape(-1, 2)
    icp = np.asarray(scene["icp_pos"], np.float64).reshape(-1, 2)
    keep = [_d(scene[k]) for k in ("uav_pos", "uav_vel", "uav_load", "tgt_pos", "tgt_vel")]
    kn, ki = _d(nfz), _d(icp)
    iv = _d(np.asarray(scene["icp_vel"], np.float64).reshape(-1, 2))
    prm = _d(params)
    p_dmg = np.zeros((N, M)); p_pen = np.zeros(N)
    lib().uo_score_pairs(N, M, len(nfz), len(icp), *[k[1] for k in keep], kn[1], ki[1], iv[1], prm[1],
                         p_dmg.ctypes.data_as(_dp), p_pen.ctypes.data_as(_dp))
    return p_dmg, p_pen


class OracleEnv:
    """One UAVEnv with an injected scene; literal restatement of uav_env.py:42-63,175-435."""

    def __init__(self, scene, params):
        self.N = len(scene["uav_load"]); self.M = len(scene["tgt_value"])
        nfz = np.asarray(scene["nfz_pos"], np.float64).reshape(-1, 2)
        icp = np.asarray(scene["icp_pos"], np.float64).reshape(-1, 2)
        self._keep = [_d(scene[k]) for k in ("uav_pos", "uav_vel", "uav_load", "uav_cost", "tgt_pos", "tgt_vel",
                                             "tgt_value")]
        tid = np.ascontiguousarray(scene["tgt_id"], dtype=np.int32)
        self._tid = tid
        extra = [_d(nfz), _d(icp), _d(np.asarray(scene["icp_vel"], np.float64).reshape(-1, 2)), _d(params)]
        self._keep += extra
        self._h = lib().uo_env_create(self.N, self.M, len(nfz), len(icp), *[k[1] for k in self._keep[:7]],
                                      tid.ctypes.data_as(_ip), *[k[1] for k in extra])
        self._obs = np.zeros((SEQ_LEN, STATE_DIM), np.float32)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().uo_env_destroy(self._h)
            self._h = None

    def reset(self):
        lib().uo_env_reset(self._h, self._obs.ctypes.data_as(_fp))
        return self._obs.copy()

    def step(self, action):
        r = ctypes.c_double(); d = ctypes.c_int(); info = np.zeros(8)
        rc = lib().uo_env_step(self._h, int(action), self._obs.ctypes.data_as(_fp), ctypes.byref(r),
                               ctypes.byref(d), info.ctypes.data_as(_dp))
        if rc != 0:
            raise IndexError("step() after the episode ended (uav_env.py:296)")
        obs = np.zeros(STATE_DIM, np.float32) if d.value else self._obs.copy()
        return obs, r.value, bool(d.value), info[:7].copy()

    @property
    def uav_idx(self):
        return lib().uo_env_uav_idx(self._h)

    @property
    def target_idx(self):
        return lib().uo_env_target_idx(self._h)

    def assigned(self):
        out = np.zeros(self.N, np.int32)
        lib().uo_env_assigned(self._h, out.ctypes.data_as(_ip))
        return out


def run_envs(envs, actions, obs_scratch=None):
    """Batched C loop (CPU baseline): actions int8 [steps, n_env]; auto state-only reset."""
    actions = np.ascontiguousarray(actions, dtype=np.int8)
    steps, n = actions.shape
    arr = (ctypes.c_void_p * n)(*[e._h for e in envs])
    scratch = np.zeros((SEQ_LEN, STATE_DIM), np.float32) if obs_scratch is None else obs_scratch
    return lib().uo_envs_run(arr, n, actions.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)), steps,
                             scratch.ctypes.data_as(_fp))
