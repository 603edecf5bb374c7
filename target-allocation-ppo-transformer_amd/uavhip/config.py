"""Constants of the reference's configs/config.py (same attribute names, same values), plus the
vectors the C ABI takes. `cfg` is the module singleton the drop-in modules share, as in the
reference (configs/config.py:88)."""
import numpy as np


class Config:
    # physics (config.py:7-12)
    PARAM_ZETA_D = 150.0
    PARAM_K = 1.2
    PARAM_C1 = 0.75
    PARAM_C2 = 0.25
    PARAM_C3 = 0.75
    PARAM_C4 = 0.25
    # weather tables (config.py:15-30; unused on the hot path)
    WEATHER_LEVEL_RANGE = (1, 6)
    WEATHER_FACTOR_TYPE1 = np.array([[0.85, 0.85, 0.85, 0.85, 0.75]] * 4 + [[0.75] * 5])
    WEATHER_FACTOR_TYPE2 = np.array([[0.9, 0.9, 0.9, 0.8, 0.8]] * 4 + [[0.8] * 5])
    # scene (config.py:33-58)
    MAP_WIDTH = 180.0
    MAP_HEIGHT = 160.0
    UAV_GEN_X_RANGE = (60, 90)
    TARGET_GEN_X_RANGE = (160, 180)
    NUM_UAVS = 30
    NUM_TARGETS = 10
    NUM_NFZ = 1
    NUM_INTERCEPTORS = 1
    INTERCEPT_RAD = 2.0
    COST_WEIGHT_OMEGA = 0.0
    WEATHER_SPEED_FACTOR = 1.0
    WEATHER_LOAD_FACTOR = 1.0
    # network / PPO (config.py:61-85)
    STATE_DIM = 14
    SEQ_LEN = 5
    ACTION_DIM = 2
    EMBED_DIM = 128
    NUM_HEADS = 8
    NUM_LAYERS = 2
    LR_ACTOR = 2e-4
    LR_CRITIC = 1e-3
    GAMMA = 0.998
    GAE_LAMBDA = 0.95
    K_EPOCHS = 5
    EPS_CLIP = 0.2
    BATCH_SIZE = 64
    GRAD_NORM_CLIP = 1.0
    MAX_EPISODES = 2000
    RESET_EPISODES = 200
    SEED = 42
    # build-side knobs (not in the reference)
    OBSTACLE_ZETA = 10.0          # mechanics.py:79
    FULL_RESET_PERIOD = 200       # main_train.py:79 `i_episode % 200 == 0`


def config0_overrides():
    """The reference's alternate "paper-original" constants (configs/config0.py)."""
    return dict(PARAM_K=5.0, UAV_GEN_X_RANGE=(0, 30), NUM_NFZ=2, NUM_INTERCEPTORS=2, INTERCEPT_RAD=3.0,
                WEATHER_SPEED_FACTOR=0.85, WEATHER_LOAD_FACTOR=0.90)


def params_vector(c):
    """include/uavhip.h UAVHIP_PRM_* vector."""
    return np.array([c.PARAM_ZETA_D, c.PARAM_K, c.PARAM_C1, c.PARAM_C2, c.PARAM_C3, c.PARAM_C4,
                     c.COST_WEIGHT_OMEGA, getattr(c, "OBSTACLE_ZETA", 10.0)], dtype=np.float64)


def gen_vector(c):
    """include/uavhip.h UAVHIP_GEN_* vector (ranges of uav_env.py:65-173)."""
    g = np.zeros(16, dtype=np.float64)
    g[0:2] = c.UAV_GEN_X_RANGE
    g[2:4] = c.TARGET_GEN_X_RANGE
    g[4] = c.MAP_HEIGHT
    g[5] = c.WEATHER_SPEED_FACTOR
    g[6] = c.WEATHER_LOAD_FACTOR
    g[7:9] = (120.0, 140.0)
    g[9:11] = (140.0, 160.0)
    g[11:13] = (0.30, 0.32)
    return g


cfg = Config()
