"""ctypes binding of libuavhip.so (C ABI declared in include/uavhip.h).

The library is built in-tree (csrc/Makefile -> uavhip/libuavhip.so). There is deliberately no
fallback: if the library is missing or cannot be loaded, importing this module raises, and every
GPU entry point raises if its HIP call fails.
"""
import ctypes
import os

# torch first: its bundled HIP runtime (libamdhip64.so.7 / libhsa-runtime64.so.1) is then the one
# libuavhip.so binds to (same sonames), so the library and torch share ONE runtime, device and set of
# streams. Loaded the other way round (the drop-in `configs` module imported before anything else,
# as main_train.py does), /opt/rocm's runtime would come in first and the two runtimes would
# contend for the device.
import torch  # noqa: F401,E402

_HERE = os.path.dirname(os.path.abspath(__file__))
# UAVHIP_LIB: an alternative in-tree build (profiling: the TRACE=1 phase-stamp build)
LIB_PATH = os.environ.get("UAVHIP_LIB") or os.path.join(_HERE, "libuavhip.so")

SEQ_LEN = 5
STATE_DIM = 14
OBS_FLOATS = SEQ_LEN * STATE_DIM
MAX_N, MAX_M, MAX_OBSTACLES = 64, 128, 8
ENV_ONE_PER_WAVE, ENV_OBS_F16, ENV_NO_REPLAY = 1, 2, 4  # uavhip_env.flags bits

PRM = dict(ZETA_D=0, K=1, C1=2, C2=3, C3=4, C4=5, OMEGA=6, ZETA_OBS=7)
PRM_COUNT = 8
GEN = dict(UAV_X0=0, UAV_X1=1, TGT_X0=2, TGT_X1=3, MAP_H=4, WEATHER_SPEED=5, WEATHER_LOAD=6, NFZ_X0=7, NFZ_X1=8,
           ICP_X0=9, ICP_X1=10, ICP_S0=11, ICP_S1=12)
GEN_COUNT = 16
INFO = dict(J=0, NUM_ASSIGNED=1, IS_VALID=2, AVG_P_DMG=3, AVG_P_FINAL=4, UAV_IDX=5, TARGET_IDX=6, EPISODE=7)
INFO_COUNT = 8
IST = dict(UAV_IDX=0, TARGET_IDX=1, N_COVERED=2, N_ASSIGNED=3, EPISODE=4, ERROR=5, SCENE_SEL=6, SCENE_STALE=7,
           SCENE_GEN=8)
IST_COUNT = 12
DST = dict(R=0, J=1, ASG_COST=2, COV_VALUE=3, TOTAL_COST=4, TOTAL_VALUE=5, PD_CUR=6, SUM_PDMG=7, SUM_PFIN=8)
DST_COUNT = 12
PPO_FORWARD, PPO_BACKWARD, PPO_UPDATE, PPO_FULL, PPO_PACKED = 1, 2, 4, 7, 8
EP = dict(ENV=0, EPISODE=1, STEPS=2, REWARD=3, Q0=4, J_SUM=5, MAX_COV=6, ACTION1=7, VALID=8, PDMG_SUM=9,
          PFINAL_SUM=10, ASSIGN_STEPS=11)
EP_COUNT = 12

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32


class EnvDesc(ctypes.Structure):
    """Mirror of `struct uavhip_env` (include/uavhip.h)."""
    _fields_ = [("E", _i32), ("N", _i32), ("M", _i32), ("Kn", _i32), ("Ki", _i32),
                ("full_reset_period", _i32), ("scene_buffers", _i32), ("flags", _i32), ("seed", ctypes.c_uint64),
                ("env_base", ctypes.c_uint64),
                ("prm", ctypes.c_double * PRM_COUNT), ("gen", ctypes.c_double * GEN_COUNT)] + \
              [(n, _vp) for n in ("uav_pos", "uav_vel", "uav_load", "uav_cost", "uav_type", "tgt_pos", "tgt_vel",
                                  "tgt_value", "tgt_id", "nfz_pos", "icp_pos", "icp_vel", "p_dmg", "p_pen",
                                  "nh_final", "nh_pure", "t_cost", "n_lock", "assigned", "istate", "dstate",
                                  "window")]


class PolicyDesc(ctypes.Structure):
    """Mirror of `struct uavhip_policy`."""
    _fields_ = [("weights", _vp), ("n_floats", _i32), ("d_model", _i32), ("n_heads", _i32), ("d_ff", _i32),
                ("d_head_hidden", _i32), ("actor_layers", _i32), ("critic_layers", _i32)]


class PPODesc(ctypes.Structure):
    """Mirror of `struct uavhip_ppo`."""
    _fields_ = [("params", _vp), ("grads", _vp), ("adam_m", _vp), ("adam_v", _vp), ("adam_step", _vp),
                ("workspace", _vp), ("loss_sums", _vp), ("stats", _vp), ("n_floats", _i32), ("minibatch", _i32),
                ("global_minibatch", _i32)] + \
              [(n, ctypes.c_double) for n in ("lr_actor", "lr_critic", "beta1", "beta2", "adam_eps")] + \
              [(n, ctypes.c_float) for n in ("eps_clip", "max_grad_norm", "value_coef", "entropy_coef")]


# name -> (restype, argtypes)
_SIGS = {
    "uavhip_score_pairs": (ctypes.c_int, [ctypes.POINTER(EnvDesc), _vp, _vp]),
    "uavhip_scene_generate": (ctypes.c_int, [ctypes.POINTER(EnvDesc), _vp, _vp]),
    "uavhip_scene_refresh": (ctypes.c_int, [ctypes.POINTER(EnvDesc), _vp]),
    "uavhip_env_reset": (ctypes.c_int, [ctypes.POINTER(EnvDesc), _vp, _i32, _vp, _vp]),
    "uavhip_env_step": (ctypes.c_int, [ctypes.POINTER(EnvDesc), _vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "uavhip_gae": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i32, _i32, ctypes.c_double, ctypes.c_double, _vp, _vp, _vp,
                                  _vp]),
    "uavhip_gae_partials": (_i32, [_i32, _i32]),
    "uavhip_adv_partials": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _i32, _vp]),
    "uavhip_adv_normalize": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _i32, ctypes.c_int64, _vp, _vp]),
    "uavhip_windows_from_rows": (ctypes.c_int, [_vp, _vp, _vp, _i32, ctypes.c_int64, _i32, _i32, _i32, _vp, _vp]),
    "uavhip_policy_layout": (_i32, [ctypes.POINTER(_i32), _i32]),
    "uavhip_policy_split_layout": (_i32, [_vp, _vp, _i32]),
    "uavhip_policy_tiling": (_i32, [ctypes.POINTER(_i32), _i32]),
    "uavhip_policy_range_table": (_i32, [_vp, _vp]),
    "uavhip_policy_pack": (ctypes.c_int, [_vp, _vp, _vp]),
    "uavhip_policy_forward": (ctypes.c_int, [ctypes.POINTER(PolicyDesc), _vp, _i32, _vp, ctypes.c_uint64,
                                             ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "uavhip_policy_rowproj_floats": (ctypes.c_int64, [_i32]),
    "uavhip_policy_forward_rows": (ctypes.c_int, [ctypes.POINTER(PolicyDesc), _vp, _i32, _vp, _i32, _i32, _vp,
                                                  ctypes.c_uint64, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp,
                                                  _vp]),
    "uavhip_policy_value_rows": (ctypes.c_int, [ctypes.POINTER(PolicyDesc), _vp, _i32, _vp, _i32, _i32, _vp, _vp]),
    "uavhip_rollout_step": (ctypes.c_int, [ctypes.POINTER(PolicyDesc), ctypes.POINTER(EnvDesc), _vp, _vp, _i32,
                                           _i32, ctypes.c_uint64, ctypes.c_uint64, _vp, _vp, _vp, _vp, _i32, _vp,
                                           _vp, _vp, _vp, _vp]),
    "uavhip_rollout_steps": (ctypes.c_int, [ctypes.POINTER(PolicyDesc), ctypes.POINTER(EnvDesc), _vp, _vp, _i32,
                                            _i32, _i32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _vp, _vp,
                                            _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "uavhip_ppo_workspace_floats": (ctypes.c_int64, [_i32]),
    "uavhip_ppo_step": (ctypes.c_int, [ctypes.POINTER(PPODesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp]),
    "uavhip_episode_stats": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _vp, _vp, _i32, _vp, _vp]),
    "uavhip_device_pci_id": (ctypes.c_int, [_i32, ctypes.c_char_p, _i32]),
    "uavhip_device_from_pci_id": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_i32)]),
    "uavhip_peer_access": (ctypes.c_int, [_i32, ctypes.POINTER(_i32)]),
    "uavhip_ipc_export": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(ctypes.c_uint64)]),
    "uavhip_ipc_open": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.POINTER(_vp)]),
    "uavhip_ipc_close": (ctypes.c_int, [_vp]),
    "uavhip_copy_async": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp]),
    "uavhip_last_error": (ctypes.c_char_p, []),
    "uavhip_abi_version": (_i32, []),
}
EXPORTS = tuple(_SIGS)


class UavHipError(RuntimeError):
    pass


ABI_VERSION = 5  # include/uavhip.h uavhip_abi_version


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libuavhip.so not built at {LIB_PATH}: run `make -C "
                          f"target-allocation-ppo-transformer_amd/csrc` (or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    # UAVHIP_ACCEPT_PREV_ABI=1 (set by the A/B timing scripts only, scripts/ab_rollout.py): an older
    # experimental build may predate an entry point and be of the previous ABI (4: no range table,
    # peers by ordinal). Anything else -- a custom UAVHIP_LIB included -- must be the current ABI with
    # every entry point, so a stale build fails here, not later and far from the cause.
    lenient = os.environ.get("UAVHIP_ACCEPT_PREV_ABI") == "1"
    missing = [name for name in _SIGS if not hasattr(lib, name)]
    if missing and not lenient:
        raise ImportError(f"{LIB_PATH}: missing entry points {missing[:4]}{'...' if len(missing) > 4 else ''}: "
                          f"rebuild (make -C target-allocation-ppo-transformer_amd/csrc)")
    for name, (res, args) in _SIGS.items():
        if name in missing:
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    ok = (ABI_VERSION, ABI_VERSION - 1) if lenient else (ABI_VERSION,)
    if lib.uavhip_abi_version() not in ok:
        raise ImportError(f"{LIB_PATH}: ABI version {lib.uavhip_abi_version()}, this binding needs {ABI_VERSION}: "
                          f"rebuild (make -C target-allocation-ppo-transformer_amd/csrc)")
    if lenient and (missing or lib.uavhip_abi_version() != ABI_VERSION):
        import warnings
        warnings.warn(f"UAVHIP_ACCEPT_PREV_ABI=1: {LIB_PATH} is ABI {lib.uavhip_abi_version()} with "
                      f"{len(missing)} entry points missing (A/B timing builds only)")
    return lib


LIB = _load()


def check(rc, what):
    if rc != 0:
        msg = LIB.uavhip_last_error().decode(errors="replace")
        raise UavHipError(f"{what} failed (rc={rc}): {msg}")


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_handle(stream=None):
    import torch
    s = torch.cuda.current_stream() if stream is None else stream
    return ctypes.c_void_p(s.cuda_stream)
