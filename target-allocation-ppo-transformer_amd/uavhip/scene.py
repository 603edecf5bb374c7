"""Host scene generator with the reference's RNG call order (envs/uav_env.py:65-173).

Used where the drop-in must reproduce the reference's scenes from the same global seeds
(`np.random.seed(s); random.seed(s)` then `UAVEnv().reset(True)` gives the same UAVs, targets and
obstacles as the reference). It draws from the GLOBAL numpy legacy stream and Python `random`,
exactly as the reference does, so it consumes those streams identically. Scene generation is not
on the per-step hot path (full resets happen every 200 episodes, main_train.py:79); the batched
rollout uses the on-device Philox generator (uavhip_scene_generate) instead.
"""
import random

import numpy as np


def generate_scene(c):
    """Returns a dict of SoA arrays in the layout of the C ABI (one env)."""
    ws, wl = c.WEATHER_SPEED_FACTOR, c.WEATHER_LOAD_FACTOR
    N, M = c.NUM_UAVS, c.NUM_TARGETS
    n_t2 = N // 4
    types = [1] * (N - n_t2) + [2] * n_t2
    random.shuffle(types)                                            # :84
    uav_pos = np.zeros((N, 2)); uav_vel = np.zeros((N, 2))
    uav_load = np.zeros(N); uav_cost = np.zeros(N); uav_max = np.zeros(N)
    total_cost = 0.0
    for i, ty in enumerate(types):                                   # :86-118
        x = np.random.uniform(c.UAV_GEN_X_RANGE[0], c.UAV_GEN_X_RANGE[1])
        y = np.random.uniform(0, c.MAP_HEIGHT)
        if ty == 1:
            base_speed, cost, base_load = np.random.uniform(0.35, 0.50), 1.0, 0.95
        else:
            base_speed, cost, base_load = np.random.uniform(0.75, 0.90), 1.25, 1.0
        speed = base_speed * ws
        ang = np.deg2rad(np.random.uniform(-15, 15))
        uav_pos[i] = (x, y)
        uav_vel[i] = np.array([np.cos(ang), np.sin(ang)]) * speed
        uav_load[i] = base_load * wl
        uav_cost[i] = cost
        uav_max[i] = speed
        total_cost += cost
    n1, n4 = M // 2, 1                                               # :121-129
    n_remain = M - n1 - n4
    n2 = np.random.randint(1, n_remain + 1) if n_remain >= 1 else 0
    n3 = n_remain - n2
    vals = [4.0] * n1 + [6.0] * n2 + [8.0] * n3 + [16.0] * n4
    random.shuffle(vals)
    tpos = np.zeros((M, 2)); tvel = np.zeros((M, 2))
    for i in range(M):                                               # :131-142
        x = np.random.uniform(c.TARGET_GEN_X_RANGE[0], c.TARGET_GEN_X_RANGE[1])
        y = np.random.uniform(0, c.MAP_HEIGHT)
        tpos[i] = (x, y)
        tvel[i] = (np.random.rand(2) - 0.5) * 0.03
    nfz_pos = np.zeros((c.NUM_NFZ, 2)); nfz_rad = np.zeros(c.NUM_NFZ)
    for i in range(c.NUM_NFZ):                                       # :147-153
        nfz_rad[i] = np.random.uniform(5, 10)
        nfz_pos[i] = (np.random.uniform(120, 140), np.random.uniform(0, c.MAP_HEIGHT))
    icp_pos = np.zeros((c.NUM_INTERCEPTORS, 2)); icp_vel = np.zeros((c.NUM_INTERCEPTORS, 2))
    for i in range(c.NUM_INTERCEPTORS):                              # :157-170
        x = np.random.uniform(140, 160)
        y = np.random.uniform(0, c.MAP_HEIGHT)
        sp = np.random.uniform(0.30, 0.32)
        a = np.random.uniform(0, 2 * np.pi)
        icp_pos[i] = (x, y)
        icp_vel[i] = np.array([np.cos(a), np.sin(a)]) * sp
    order = np.arange(M)
    # np.random.shuffle(self.targets) (:173): shuffling a list of objects with the legacy
    # generator permutes exactly like shuffling an index array of the same length.
    np.random.shuffle(order)
    return dict(uav_pos=uav_pos, uav_vel=uav_vel, uav_load=uav_load, uav_cost=uav_cost,
                uav_type=np.array(types, np.int32), uav_maxspeed=uav_max,
                tgt_pos=tpos[order], tgt_vel=tvel[order], tgt_value=np.array(vals)[order],
                tgt_id=order.astype(np.int32), nfz_pos=nfz_pos, nfz_radius=nfz_rad,
                icp_pos=icp_pos, icp_vel=icp_vel, icp_radius=np.full(c.NUM_INTERCEPTORS, c.INTERCEPT_RAD),
                total_swarm_cost=total_cost)
