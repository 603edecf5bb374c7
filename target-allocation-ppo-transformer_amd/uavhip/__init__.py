"""uavhip -- MI355X-native (gfx950) PPO rollout hot path of the UAV->target allocation reference.

    VecUAVEnv          E envs resident in HBM, stepped by HIP kernels (env.hip)
    TransformerActorCritic  reference-compatible policy; fused forward (policy.hip): fp32-accurate split
                       products on the f16 MFMA, embeddings and heads on the f32 MFMA
    gae                GAE + advantage normalisation on the GPU (gae.hip)
    RolloutEngine      T-step batched rollout (+ RCCL trajectory all-gather)
    PPOAgent           agents/ppo.py API
    load_checkpoint    the reference's torch.save(state_dict) files, older architectures reported

Importing this package loads libuavhip.so and raises if it is missing: there is no CPU fallback.
"""
from ._lib import LIB, UavHipError  # noqa: F401  (loads the HIP library or raises)
from .checkpoint import load_checkpoint, save_checkpoint  # noqa: F401
from .config import Config, cfg  # noqa: F401
from .policy import TransformerActorCritic, pack_weights  # noqa: F401
from .ppo import PPOAgent, gae  # noqa: F401
from .rollout import RolloutEngine, Trajectory  # noqa: F401
from .vec_env import VecUAVEnv  # noqa: F401

__all__ = ["LIB", "UavHipError", "Config", "cfg", "TransformerActorCritic", "pack_weights", "PPOAgent", "gae",
           "RolloutEngine", "Trajectory", "VecUAVEnv", "load_checkpoint", "save_checkpoint"]
