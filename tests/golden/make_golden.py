#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Test infrastructure only: this script runs in the build container (where
/root/reference is mounted read-only), never on the GPU box and never from the
product package.  It imports the reference's own modules through the 3-name
`gym` stub in tests/golden/gym_stub (gym is not installed here; the reference
only subclasses gym.Env and builds two space objects, `envs/uav_env.py:2,6,13-24`).

Outputs (all numpy .npz, loaded with allow_pickle=False):
  mechanics.npz  scalar KATs for envs/mechanics.py (angle/speed/dist/damage/penetration),
                 incl. the three check_reward_mechanics.py scenarios
  scenes.npz     scenes (SoA) + dense p_dmg/p_pen/p_final tables (calc_advantage per pair)
  traj.npz       (scene, action sequence) -> per-step obs/reward/done/ptr/assigned/info,
                 several episodes per case (1 full reset + state-only resets),
                 for config.py and config0.py constants, omega 0 and 0.5
  policy.npz     TransformerActorCritic state_dicts + state batch -> logits/logp/value/entropy
  gae.npz        PPOAgent.update() GAE returns + normalised advantages (captured in-frame)
  ppo_update.npz one full PPOAgent.update() (seeded sampler) -> losses + final weights
  main_train.npz main_train.train() itself for 30 episodes: every env.step (action, reward, done,
                 info), the per-episode statistic accumulators of main_train.py:98-136 read from
                 train()'s own frame, its CSV rows (:161-195) and the update losses behind them
  init_rng.npz   the sampler's first torch.randperm after PPOAgent() / two networks under
                 torch.manual_seed (the CPU generator's position after construction)

Usage:  python tests/golden/make_golden.py   (takes ~1 min on CPU; `... init_rng` writes only init_rng.npz)
"""
import json
import os
import random
import sys

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("UAV_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(HERE, "gym_stub"))
sys.path.insert(1, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from configs.config import cfg  # noqa: E402
import configs.config0 as config0  # noqa: E402
import envs.mechanics as mech  # noqa: E402
from envs.entities import UAV, Target, NoFlyZone, Interceptor  # noqa: E402
from envs.uav_env import UAVEnv  # noqa: E402
from networks.transformer_net import TransformerActorCritic  # noqa: E402
from agents.ppo import PPOAgent  # noqa: E402

CFG_KEYS = ["PARAM_ZETA_D", "PARAM_K", "PARAM_C1", "PARAM_C2", "PARAM_C3", "PARAM_C4",
            "MAP_WIDTH", "MAP_HEIGHT", "UAV_GEN_X_RANGE", "TARGET_GEN_X_RANGE",
            "NUM_UAVS", "NUM_TARGETS", "NUM_NFZ", "NUM_INTERCEPTORS", "INTERCEPT_RAD",
            "COST_WEIGHT_OMEGA", "WEATHER_SPEED_FACTOR", "WEATHER_LOAD_FACTOR"]
BASE_A = {k: getattr(cfg, k) for k in CFG_KEYS}
BASE_0 = {k: getattr(config0.cfg, k) for k in CFG_KEYS}


def apply_cfg(base, **over):
    d = dict(base)
    d.update(over)
    for k, v in d.items():
        setattr(cfg, k, v)
    return d


def meta():
    return {"numpy": np.__version__, "torch": torch.__version__, "python": sys.version.split()[0],
            "reference": REF}


def params_vec(d):
    """The constant vector the build's C-ABI takes (include/uavhip.h UAV_PARAM_*)."""
    return np.array([d["PARAM_ZETA_D"], d["PARAM_K"], d["PARAM_C1"], d["PARAM_C2"],
                     d["PARAM_C3"], d["PARAM_C4"], d["COST_WEIGHT_OMEGA"], 10.0], dtype=np.float64)


# ----------------------------------------------------------------------------- mechanics
def gen_mechanics(rng):
    out = {}
    K = 600
    up = rng.uniform(0, 180, size=(K, 2))
    uv = rng.normal(size=(K, 2)) * rng.uniform(0, 1, size=(K, 1))
    tp = rng.uniform(0, 180, size=(K, 2))
    # edge cases: coincident point, zero velocity, tiny distance (b clamp), collinear +/-.
    tp[0] = up[0]
    uv[1] = 0.0
    tp[2] = up[2] + np.array([3e-4, 1e-4])
    uv[3] = np.array([0.5, 0.0]); tp[3] = up[3] + np.array([10.0, 0.0])
    uv[4] = np.array([0.5, 0.0]); tp[4] = up[4] - np.array([10.0, 0.0])
    uv[5] = np.array([1e-7, 0.0])
    tp[6] = up[6] + np.array([5e-7, 0.0])
    tp[7:40] = up[7:40] + rng.normal(size=(33, 2)) * 0.01
    ang = np.array([mech.calc_angle_score(up[i], uv[i], tp[i]) for i in range(K)], dtype=np.float64)
    out.update(ang_uav_pos=up, ang_uav_vel=uv, ang_pt=tp, ang_out=ang)

    us = rng.uniform(0, 1, size=K); ts = rng.uniform(0, 0.9, size=K)
    us[0] = 0.0; us[1] = 5e-7; ts[2] = 0.0; us[3] = ts[3] * 1.2
    sp = np.array([mech.calc_speed_score(us[i], ts[i]) for i in range(K)], dtype=np.float64)
    out.update(spd_u=us, spd_t=ts, spd_out=sp)

    d = rng.uniform(0, 300, size=K); d[0] = 0.0
    out.update(dst_d=d,
               dst_tgt=np.array([mech.calc_dist_score(x, False) for x in d], dtype=np.float64),
               dst_obs=np.array([mech.calc_dist_score(x, True) for x in d], dtype=np.float64))

    # damage / penetration / advantage on random records (loads up to 1.3 so the clip fires).
    P = 400
    recs = dict(u_pos=rng.uniform([40, 0], [100, 160], size=(P, 2)),
                u_vel=rng.normal(size=(P, 2)) * 0.5,
                u_load=rng.uniform(0.5, 1.3, size=P),
                t_pos=rng.uniform([100, 0], [180, 160], size=(P, 2)),
                t_vel=(rng.uniform(size=(P, 2)) - 0.5) * 0.6,
                n_pos=rng.uniform([90, 0], [150, 160], size=(P, 2, 2)),
                i_pos=rng.uniform([90, 0], [160, 160], size=(P, 2, 2)),
                i_vel=rng.normal(size=(P, 2, 2)) * 0.3,
                kn=rng.integers(0, 3, size=P), ki=rng.integers(0, 3, size=P))
    recs["u_vel"][0] = 0.0
    recs["t_pos"][1] = recs["u_pos"][1]
    recs["n_pos"][2, 0] = recs["u_pos"][2]
    recs["i_pos"][3, 0] = recs["u_pos"][3] + np.array([1e-3, 0.0])
    dmg, pen, fin = [], [], []
    for i in range(P):
        u = UAV(id=0, pos=recs["u_pos"][i], velocity=recs["u_vel"][i], max_speed=0.0, load=recs["u_load"][i])
        t = Target(id=0, pos=recs["t_pos"][i], value=4.0)
        t.velocity = recs["t_vel"][i]
        nf = [NoFlyZone(id=j, pos=recs["n_pos"][i, j], radius=5.0) for j in range(recs["kn"][i])]
        it = []
        for j in range(recs["ki"][i]):
            x = Interceptor(id=j, pos=recs["i_pos"][i, j], radius=2.0)
            x.velocity = recs["i_vel"][i, j]
            it.append(x)
        dmg.append(mech.calc_damage_prob(u, t))
        pen.append(mech.calc_penetration_prob(u, t, nf, it))
        fin.append(mech.calc_advantage(u, t, nf, it)[0])
    for k, v in recs.items():
        out["rec_" + k] = v
    out.update(rec_dmg=np.array(dmg, np.float64), rec_pen=np.array(pen, np.float64),
               rec_fin=np.array(fin, np.float64))

    # check_reward_mechanics.py:80-106 scenarios (uav at origin, target at (d,0), heading angle).
    kat = []
    for dist_km, angle_deg in [(140.0, 10.0), (80.0, 5.0), (20.0, 2.0)]:
        th = np.deg2rad(angle_deg)
        u = UAV(id=0, pos=np.array([0.0, 0.0]), velocity=np.array([np.cos(th), np.sin(th)]) * 0.4,
                max_speed=0.4, load=1.0)
        t = Target(id=0, pos=np.array([float(dist_km), 0.0]), value=4.0)
        t.velocity = np.array([-1.0, 0.0]) * 0.01
        kat.append([dist_km, angle_deg, mech.calc_dist_score(dist_km, False),
                    mech.calc_angle_score(u.pos, u.velocity, t.pos),
                    mech.calc_speed_score(np.linalg.norm(u.velocity), 0.01), mech.calc_damage_prob(u, t)])
    out["kat_check_reward"] = np.array(kat, np.float64)
    out["params"] = params_vec(BASE_A)
    return out


# ----------------------------------------------------------------------------- scenes
def extract_scene(env):
    u = env.uavs
    t = env.targets
    s = dict(
        uav_pos=np.array([x.pos for x in u], np.float64).reshape(-1, 2),
        uav_vel=np.array([x.velocity for x in u], np.float64).reshape(-1, 2),
        uav_load=np.array([x.load for x in u], np.float64),
        uav_cost=np.array([x.cost for x in u], np.float64),
        uav_type=np.array([x.uav_type for x in u], np.int32),
        uav_maxspeed=np.array([x.max_speed for x in u], np.float64),
        tgt_pos=np.array([x.pos for x in t], np.float64).reshape(-1, 2),
        tgt_vel=np.array([x.velocity for x in t], np.float64).reshape(-1, 2),
        tgt_value=np.array([x.value for x in t], np.float64),
        tgt_id=np.array([x.id for x in t], np.int32),
        nfz_pos=np.array([x.pos for x in env.nfz_list], np.float64).reshape(-1, 2),
        nfz_radius=np.array([x.radius for x in env.nfz_list], np.float64),
        icp_pos=np.array([x.pos for x in env.interceptors], np.float64).reshape(-1, 2),
        icp_vel=np.array([x.velocity for x in env.interceptors], np.float64).reshape(-1, 2),
        icp_radius=np.array([x.radius for x in env.interceptors], np.float64),
    )
    N, M = len(u), len(t)
    p_fin = np.zeros((N, M)); p_dmg = np.zeros((N, M)); p_pen = np.zeros(N)
    for i, uu in enumerate(u):
        p_pen[i] = mech.calc_penetration_prob(uu, t[0], env.nfz_list, env.interceptors)
        for j, tt in enumerate(t):
            p_fin[i, j], p_dmg[i, j] = mech.calc_advantage(uu, tt, env.nfz_list, env.interceptors)
    s.update(p_final=p_fin, p_dmg=p_dmg, p_pen=p_pen)
    return s


def gen_scenes():
    out = {}
    cases = []
    for (N, M, seeds, base, name) in [(16, 32, range(8), BASE_A, "A"), (64, 128, range(3), BASE_A, "A"),
                                      (8, 16, range(4), BASE_0, "0"), (30, 10, range(2), BASE_A, "A")]:
        for s in seeds:
            d = apply_cfg(base, NUM_UAVS=N, NUM_TARGETS=M)
            np.random.seed(s); random.seed(s)
            env = UAVEnv()
            env.reset(full_reset=True)
            sc = extract_scene(env)
            key = f"c{len(cases)}"
            for k, v in sc.items():
                out[f"{key}/{k}"] = v
            out[f"{key}/params"] = params_vec(d)
            cases.append(dict(key=key, cfg=name, N=N, M=M, seed=s))
    apply_cfg(BASE_A)
    out["manifest"] = np.array(json.dumps(dict(cases=cases, meta=meta())))
    return out


# ----------------------------------------------------------------------------- trajectories
def run_traj(base, cfgname, N, M, seed, omega, n_eps, p_assign):
    d = apply_cfg(base, NUM_UAVS=N, NUM_TARGETS=M, COST_WEIGHT_OMEGA=omega)
    np.random.seed(seed); random.seed(seed)
    env = UAVEnv()
    rs = np.random.RandomState(1000 + seed)
    rec = {k: [] for k in ["action", "obs", "terminal_obs_zero", "reward", "done", "uav_idx", "target_idx",
                           "assigned", "J_val", "num_assigned", "is_valid", "avg_p_dmg", "avg_p_final",
                           "episode"]}
    reset_obs = []
    scene = None
    for ep in range(n_eps):
        obs = env.reset(full_reset=(ep == 0))
        if ep == 0:
            scene = extract_scene(env)
        reset_obs.append(np.asarray(obs, np.float32))
        done = False
        while not done:
            a = int(rs.randint(2)) if p_assign == 0.5 else int(rs.rand() < p_assign)
            obs, r, done, info = env.step(a)
            obs = np.asarray(obs)
            rec["action"].append(a)
            if done:
                assert obs.shape == (cfg.STATE_DIM,) and not obs.any()
                rec["obs"].append(np.zeros((cfg.SEQ_LEN, cfg.STATE_DIM), np.float32))
                rec["terminal_obs_zero"].append(1)
            else:
                rec["obs"].append(obs.astype(np.float32))
                rec["terminal_obs_zero"].append(0)
            rec["reward"].append(float(r))
            rec["done"].append(int(done))
            rec["uav_idx"].append(env.uav_idx)
            rec["target_idx"].append(env.target_idx)
            rec["assigned"].append([x.assigned_target_id for x in env.uavs])
            rec["J_val"].append(info["J_val"])
            rec["num_assigned"].append(info["num_assigned"])
            iv = info["is_valid_action"]
            rec["is_valid"].append(-1 if iv is None else int(bool(iv)))
            rec["avg_p_dmg"].append(info["avg_p_dmg"])
            rec["avg_p_final"].append(info["avg_p_final"])
            rec["episode"].append(ep)
    out = {k: np.asarray(v) for k, v in rec.items()}
    out["reward"] = out["reward"].astype(np.float64)
    out["obs"] = out["obs"].astype(np.float32)
    out["reset_obs"] = np.stack(reset_obs).astype(np.float32)
    out["assigned"] = out["assigned"].astype(np.int32)
    for k in ["J_val", "avg_p_dmg", "avg_p_final"]:
        out[k] = out[k].astype(np.float64)
    for k, v in scene.items():
        out[k] = v
    out["params"] = params_vec(d)
    out["total_swarm_cost"] = np.float64(env.total_swarm_cost)
    apply_cfg(BASE_A)
    return out


def gen_traj():
    out = {}
    cases = []
    plan = []
    plan += [(BASE_A, "A", 4, 4, s, 0.0, 3, 0.5) for s in range(10)]
    plan += [(BASE_A, "A", 8, 16, s, 0.0, 3, 0.5) for s in range(5)]
    plan += [(BASE_A, "A", 16, 32, s, 0.0, 3, 0.5) for s in range(4)]
    plan += [(BASE_A, "A", 30, 10, s, 0.0, 2, 0.5) for s in range(3)]
    plan += [(BASE_A, "A", 64, 128, 0, 0.0, 1, 0.5)]
    plan += [(BASE_A, "A", 4, 4, s, 0.5, 3, 0.5) for s in range(5)]
    plan += [(BASE_A, "A", 8, 16, s, 0.5, 3, 0.5) for s in range(3)]
    plan += [(BASE_A, "A", 16, 32, 0, 2.0, 2, 0.5)]
    plan += [(BASE_0, "0", 4, 4, s, 0.0, 3, 0.5) for s in range(5)]
    plan += [(BASE_0, "0", 8, 16, s, 0.0, 3, 0.5) for s in range(3)]
    plan += [(BASE_A, "A", 4, 4, s, 0.0, 3, 0.1) for s in range(5)]
    plan += [(BASE_A, "A", 8, 16, s, 0.0, 2, 0.1) for s in range(2)]
    plan += [(BASE_A, "A", 16, 32, 1, 0.0, 2, 0.9)]
    for (base, name, N, M, s, omega, neps, pa) in plan:
        r = run_traj(base, name, N, M, s, omega, neps, pa)
        key = f"c{len(cases)}"
        for k, v in r.items():
            out[f"{key}/{k}"] = v
        cases.append(dict(key=key, cfg=name, N=N, M=M, seed=s, omega=omega, episodes=neps, p_assign=pa,
                          steps=int(len(r["action"]))))
    out["manifest"] = np.array(json.dumps(dict(cases=cases, meta=meta())))
    return out


# ----------------------------------------------------------------------------- policy
def policy_states(rng, traj):
    keys = [c["key"] for c in json.loads(str(traj["manifest"]))["cases"]]
    pool = []
    for k in keys:
        pool.append(traj[f"{k}/reset_obs"])
        ob = traj[f"{k}/obs"]
        pool.append(ob[traj[f"{k}/terminal_obs_zero"] == 0])
    pool = np.concatenate(pool)
    idx = rng.choice(len(pool), size=192, replace=False)
    real = pool[idx]
    syn = (rng.normal(size=(64, 5, 14)) * 0.7).astype(np.float32)
    for i in range(64):
        z = i % 8
        if z < 5:
            syn[i, :z] = 0.0           # prefix padding of z rows
        elif z == 5:
            syn[i, 2] = 0.0            # interior zero row (masked too: mask is per-row)
        elif z == 6:
            syn[i, -1] = 0.0           # zero last row is never masked (transformer_net.py:54)
        else:
            syn[i, :4] = 0.0; syn[i, -1] = 0.0
    return np.concatenate([real, syn]).astype(np.float32)


def policy_outputs(net, states, actions):
    with torch.no_grad():
        x = torch.from_numpy(states)
        a = torch.from_numpy(actions)
        logp, value, ent = net.evaluate(x, a)
        h = net.actor_net(x)[:, -1, :]
        logits = net.actor_head(h)
        _, _, v2, _ = net.get_action(x)
    return dict(logits=logits.numpy(), logp=logp.numpy(), value=value.numpy().reshape(-1),
                entropy=ent.numpy(), value_get_action=v2.numpy().reshape(-1))


def gen_policy(traj):
    rng = np.random.default_rng(7)
    out = {}
    states = policy_states(rng, traj)
    actions = rng.integers(0, 2, size=len(states)).astype(np.int64)
    out["states"] = states
    out["actions"] = actions
    torch.manual_seed(0)
    net_a = TransformerActorCritic()
    torch.manual_seed(1)
    net_b = TransformerActorCritic()
    with torch.no_grad():  # make every layer distinct (deepcopy makes them identical at init)
        for p in net_b.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    for tag, net in [("a", net_a), ("b", net_b)]:
        assert net.training  # the reference never calls .eval() on policy_old (ppo.py:55)
        for k, v in net.state_dict().items():
            out[f"{tag}/w/{k}"] = v.detach().numpy().copy()
        for k, v in policy_outputs(net, states, actions).items():
            out[f"{tag}/{k}"] = v
    out["keys"] = np.array(json.dumps(list(net_a.state_dict().keys())))
    out["nparams"] = np.int64(sum(p.numel() for p in net_a.parameters()))
    out["meta"] = np.array(json.dumps(meta()))
    return out


# ----------------------------------------------------------------------------- GAE
class _Captured(Exception):
    pass


def capture_gae(rewards, dones, values):
    agent = PPOAgent()
    T = len(rewards)
    for t in range(T):
        agent.buffer["states"].append(torch.zeros(1, 5, 14))
        agent.buffer["actions"].append(torch.zeros(1, dtype=torch.int64))
        agent.buffer["logprobs"].append(torch.zeros(1))
        agent.buffer["values"].append(torch.tensor([[values[t]]], dtype=torch.float32))
        agent.store_transition(float(rewards[t]), bool(dones[t]))
    box = {}

    def spy(states, actions):
        f = sys._getframe(1)
        box["returns"] = f.f_locals["returns"].detach().numpy().copy()
        box["advantages"] = f.f_locals["advantages"].detach().numpy().copy()
        raise _Captured()

    agent.policy.evaluate = spy
    try:
        agent.update()
    except _Captured:
        pass
    return box["returns"], box["advantages"]


def gen_gae():
    rng = np.random.default_rng(11)
    out = {}
    cases = []
    for T in [64, 256, 1000, 2048]:
        lens = []
        while sum(lens) < T:
            lens.append(int(rng.integers(2, 60)))
        lens[-1] -= sum(lens) - T
        if lens[-1] < 1:
            lens.pop(); lens[-1] += T - sum(lens)
        dones = np.zeros(T, np.int8)
        dones[np.cumsum(lens) - 1] = 1
        rewards = np.where(rng.uniform(size=T) < 0.5, 0.0, rng.uniform(0, 3, size=T)).astype(np.float64)
        rewards[dones == 1] += rng.uniform(5, 40, size=int(dones.sum()))
        values = (rng.normal(size=T) * 4).astype(np.float32)
        ret, adv = capture_gae(rewards, dones, values)
        key = f"c{len(cases)}"
        out.update({f"{key}/rewards": rewards, f"{key}/dones": dones, f"{key}/values": values,
                    f"{key}/returns": ret, f"{key}/advantages": adv})
        cases.append(dict(key=key, T=T))
    out["manifest"] = np.array(json.dumps(dict(cases=cases, gamma=cfg.GAMMA, lam=cfg.GAE_LAMBDA, meta=meta())))
    return out


# ----------------------------------------------------------------------------- PPO update
def gen_update(policy):
    rng = np.random.default_rng(5)
    torch.manual_seed(0)
    agent = PPOAgent()
    T = 192
    states = policy["states"][:T]
    with torch.no_grad():
        acts, lps, vals = [], [], []
        for t in range(T):
            torch.manual_seed(100 + t)
            a, lp, v, _ = agent.policy_old.get_action(torch.from_numpy(states[t:t + 1]))
            acts.append(a); lps.append(lp); vals.append(v)
    dones = np.zeros(T, np.int8)
    dones[[30, 70, 71, 130, T - 1]] = 1
    rewards = np.where(rng.uniform(size=T) < 0.5, 0.0, rng.uniform(0, 2, size=T))
    for t in range(T):
        agent.buffer["states"].append(torch.from_numpy(states[t:t + 1]))
        agent.buffer["actions"].append(acts[t])
        agent.buffer["logprobs"].append(lps[t])
        agent.buffer["values"].append(vals[t])
        agent.store_transition(float(rewards[t]), bool(dones[t]))
    out = {"states": states, "actions": torch.cat(acts).numpy(), "logprobs": torch.cat(lps).numpy(),
           "values": torch.cat(vals).numpy().reshape(-1), "rewards": rewards, "dones": dones}
    for k, v in agent.policy.state_dict().items():
        out["w0/" + k] = v.numpy().copy()
    # record the sampler's index stream so a build can replay the same minibatches
    torch.manual_seed(1234)
    perms = [torch.randperm(T).numpy() for _ in range(cfg.K_EPOCHS)]
    torch.manual_seed(1234)
    stats = agent.update()
    out["perms"] = np.stack(perms).astype(np.int64)
    out["loss_actor"] = np.float64(stats["loss_actor"])
    out["loss_critic"] = np.float64(stats["loss_critic"])
    out["entropy"] = np.float64(stats["entropy"])
    for k, v in agent.policy.state_dict().items():
        out["w1/" + k] = v.numpy().copy()
    out["meta"] = np.array(json.dumps(meta()))
    return out


# ----------------------------------------------------------------------------- CPU RNG after init
def gen_init_rng():
    """The sampler's first permutation (SubsetRandomSampler -> torch.randperm, ppo.py:115) drawn right
    after building the networks under torch.manual_seed(s): PPOAgent() builds policy and policy_old
    (ppo.py:13-43). A build whose construction draws anything extra from the CPU generator shifts it."""
    out = {}
    for s in (0, 7):
        torch.manual_seed(s)
        TransformerActorCritic()
        TransformerActorCritic()
        out[f"two_nets/{s}"] = torch.randperm(192).numpy()
        torch.manual_seed(s)
        PPOAgent()
        out[f"agent/{s}"] = torch.randperm(192).numpy()
    out["meta"] = np.array(json.dumps(meta()))
    return out


# ----------------------------------------------------------------------------- main_train statistics
EP_LOCALS = ("current_ep_reward", "current_q0", "ep_total_J", "ep_steps", "ep_max_cov", "ep_action1_cnt",
             "ep_valid_cnt", "ep_total_p_dmg", "ep_total_p_final", "ep_steps_with_assign")


def gen_main_train(episodes=30):
    """Run the reference's training driver (main_train.train) and record what its statistics are
    made of and what it computed from them: env.step is wrapped to log each step's action / reward /
    done / info; the per-episode accumulators are read from train()'s own frame when the next
    episode's env.reset() is called (and, for the last episode, when its CSV row is written); the
    CSV writer is wrapped to capture the rows and the update stats behind their loss columns."""
    import csv
    import tempfile
    import main_train as mt
    steps, eps, rows = [], [], []
    real_step, real_reset, real_writer = UAVEnv.step, UAVEnv.reset, csv.writer

    def frame_of_train():
        f = sys._getframe(2)
        return f.f_locals if f.f_code.co_name == "train" else None

    def snapshot(fl, episode):
        return [float(episode)] + [float(fl[k]) for k in EP_LOCALS]

    def step(self, action):
        obs, r, d, info = real_step(self, action)
        iv = info["is_valid_action"]
        steps.append([len(eps) + 1, action, r, float(d), info["J_val"], info["num_assigned"],
                      -1.0 if iv is None else float(bool(iv)), info["avg_p_dmg"], info["avg_p_final"]])
        return obs, r, d, info

    def reset(self, full_reset=True):
        fl = frame_of_train()
        if fl is not None and "ep_total_J" in fl:   # the previous episode's final accumulators
            eps.append(snapshot(fl, fl["i_episode"] - 1))
        return real_reset(self, full_reset)

    class Writer:
        def __init__(self, f):
            self.w = real_writer(f)

        def writerow(self, row):
            fl = sys._getframe(1).f_locals
            if "ep_total_J" in fl:
                st = fl["ppo_stats"]
                rows.append(([str(x) for x in row], [st["loss_critic"], st["loss_actor"], st["entropy"]] if st else
                             [0.0, 0.0, 0.0]))
                if fl["i_episode"] == episodes:
                    eps.append(snapshot(fl, fl["i_episode"]))
            return self.w.writerow(row)

    saved = (cfg.MAX_EPISODES, os.getcwd())
    UAVEnv.step, UAVEnv.reset, csv.writer = step, reset, Writer
    try:
        cfg.MAX_EPISODES = episodes
        np.random.seed(0); random.seed(0); torch.manual_seed(0)
        with tempfile.TemporaryDirectory() as d:
            os.chdir(d)
            mt.train()
    finally:
        UAVEnv.step, UAVEnv.reset, csv.writer = real_step, real_reset, real_writer
        cfg.MAX_EPISODES = saved[0]
        os.chdir(saved[1])
    assert len(eps) == episodes and len(rows) == episodes // 10
    return {"steps": np.array(steps, np.float64), "episodes": np.array(eps, np.float64),
            "csv_rows": np.array(json.dumps([r for r, _ in rows])),
            "csv_losses": np.array([l for _, l in rows], np.float64),
            "fields": np.array(json.dumps(["episode", "action", "reward", "done", "J_val", "num_assigned", "is_valid",
                                           "avg_p_dmg", "avg_p_final"])),
            "episode_fields": np.array(json.dumps(["episode"] + list(EP_LOCALS))), "meta": np.array(json.dumps(meta()))}


def main():
    outdir = HERE
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if sys.argv[1:] == ["init_rng"]:  # the one fixture added in round 3
        np.savez_compressed(os.path.join(outdir, "init_rng.npz"), **gen_init_rng())
        return
    np.savez_compressed(os.path.join(outdir, "mechanics.npz"), **gen_mechanics(np.random.default_rng(3)))
    np.savez_compressed(os.path.join(outdir, "scenes.npz"), **gen_scenes())
    traj = gen_traj()
    np.savez_compressed(os.path.join(outdir, "traj.npz"), **traj)
    pol = gen_policy(traj)
    np.savez_compressed(os.path.join(outdir, "policy.npz"), **pol)
    np.savez_compressed(os.path.join(outdir, "gae.npz"), **gen_gae())
    np.savez_compressed(os.path.join(outdir, "ppo_update.npz"), **gen_update(pol))
    np.savez_compressed(os.path.join(outdir, "main_train.npz"), **gen_main_train())
    print("golden fixtures written to", outdir)


if __name__ == "__main__":
    main()
