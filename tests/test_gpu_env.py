"""GPU parity of the env kernels (K1 score_pairs, reset, K2 step, on-device scene generation)
against the reference's golden vectors and the CPU oracle. Marked gpu; run with -m gpu.

Bars: allocation indices / pointer walk / done / num_assigned / is_valid bit-exact; pair
probabilities to ulp level (ocml vs glibc acos/exp); rewards and info to 1e-9 relative; obs windows
to 2e-6 (fp32 cast of fp64 features; almost all windows bit-identical)."""
import numpy as np
import pytest
import torch

from conftest import cases, has_gpu, sub

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]

RTOL_P, ATOL_P = 5e-12, 1e-15


def _venv(E, N, M, Kn, Ki, params=None, period=0, seed=0):
    from uavhip.vec_env import VecUAVEnv
    v = VecUAVEnv(E, N, M, Kn, Ki, full_reset_period=period, seed=seed)
    if params is not None:
        v.set_params(params)
    return v


def test_score_pairs_vs_reference(scenes_npz):
    groups = {}
    for c in cases(scenes_npz):
        s = sub(scenes_npz, c["key"])
        key = (c["N"], c["M"], len(s["nfz_pos"]), len(s["icp_pos"]), tuple(s["params"]))
        groups.setdefault(key, []).append(s)
    for (N, M, Kn, Ki, prm), ss in groups.items():
        v = _venv(len(ss), N, M, Kn, Ki, np.array(prm))
        v.load_scenes(ss)
        torch.cuda.synchronize()
        p_dmg, p_pen = v.p_dmg.cpu().numpy(), v.p_pen.cpu().numpy()
        for i, s in enumerate(ss):
            np.testing.assert_allclose(p_dmg[i], s["p_dmg"], rtol=RTOL_P, atol=ATOL_P)
            np.testing.assert_allclose(p_pen[i], s["p_pen"], rtol=RTOL_P, atol=ATOL_P)
            np.testing.assert_allclose(p_dmg[i] * p_pen[i][:, None], s["p_final"], rtol=RTOL_P, atol=ATOL_P)


def test_mechanics_records_vs_reference(mech_npz):
    """envs/mechanics.py KATs incl. edge cases (zero velocity, coincident points, clip) via K1 with
    one UAV and one target per env."""
    d = mech_npz
    P = len(d["rec_dmg"])
    for kn in range(3):
        for ki in range(3):
            idx = [i for i in range(P) if d["rec_kn"][i] == kn and d["rec_ki"][i] == ki]
            if not idx:
                continue
            v = _venv(len(idx), 1, 1, kn, ki, d["params"])
            scenes = []
            for i in idx:
                scenes.append(dict(uav_pos=d["rec_u_pos"][i], uav_vel=d["rec_u_vel"][i], uav_load=[d["rec_u_load"][i]],
                                   uav_cost=[1.0], tgt_pos=d["rec_t_pos"][i], tgt_vel=d["rec_t_vel"][i],
                                   tgt_value=[4.0], tgt_id=[0], nfz_pos=d["rec_n_pos"][i][:kn],
                                   icp_pos=d["rec_i_pos"][i][:ki], icp_vel=d["rec_i_vel"][i][:ki]))
            v.load_scenes(scenes)
            np.testing.assert_allclose(v.p_dmg.cpu().numpy().reshape(-1), d["rec_dmg"][idx], rtol=RTOL_P, atol=ATOL_P)
            np.testing.assert_allclose(v.p_pen.cpu().numpy().reshape(-1), d["rec_pen"][idx], rtol=RTOL_P, atol=ATOL_P)


def _check_traj(got, s, rtol_r=1e-9):
    np.testing.assert_array_equal(got["done"], s["done"])
    np.testing.assert_array_equal(got["uav_idx"], s["uav_idx"])
    np.testing.assert_array_equal(got["target_idx"], s["target_idx"])
    np.testing.assert_array_equal(got["assigned"], s["assigned"])
    np.testing.assert_array_equal(got["num_assigned"], s["num_assigned"])
    np.testing.assert_array_equal(got["is_valid"], s["is_valid"])
    scale = np.maximum(np.abs(s["reward"]), 1e-3)
    assert np.max(np.abs(got["reward"] - s["reward"]) / scale) < rtol_r
    np.testing.assert_allclose(got["J_val"], s["J_val"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(got["avg_p_dmg"], s["avg_p_dmg"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(got["avg_p_final"], s["avg_p_final"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(got["obs"], s["obs"], rtol=2e-6, atol=1e-6)


def _replay_batched(group, fused=False):
    """Replay every case of `group` (same dims/params) in ONE VecUAVEnv, one env per case,
    stepping all envs together; episodes restart with a state-only reset (host-driven)."""
    from uavhip import _lib
    s0 = group[0]
    N, M = len(s0["uav_load"]), len(s0["tgt_value"])
    v = _venv(len(group), N, M, len(s0["nfz_pos"]), len(s0["icp_pos"]), s0["params"])
    v.load_scenes(group)
    E = len(group)
    res = [dict(obs=[], reward=[], done=[], uav_idx=[], target_idx=[], assigned=[], J_val=[], num_assigned=[],
                is_valid=[], avg_p_dmg=[], avg_p_final=[], reset_obs=[]) for _ in range(E)]
    # per env list of episodes of actions
    eps = []
    for s in group:
        ep_actions = []
        for ep in range(int(s["episode"].max()) + 1):
            ep_actions.append(s["action"][s["episode"] == ep])
        eps.append(ep_actions)
    n_eps = max(len(x) for x in eps)
    for ep in range(n_eps):
        obs0 = v.reset(episode=ep + 1).cpu().numpy()
        for e in range(E):
            if ep < len(eps[e]):
                res[e]["reset_obs"].append(obs0[e])
        L = max(len(eps[e][ep]) if ep < len(eps[e]) else 0 for e in range(E))
        acts = np.zeros((L, E), np.int8)
        for e in range(E):
            if ep < len(eps[e]):
                acts[:len(eps[e][ep]), e] = eps[e][ep]
        A = torch.as_tensor(acts, device="cuda")
        if fused:
            obs, rew, done, info = v.step(A, auto_reset=False)
            outs = [(obs[t].cpu().numpy(), rew[t].cpu().numpy(), done[t].cpu().numpy(), info[t].cpu().numpy(),
                     None) for t in range(L)]
            asg_final = v.assigned_target_ids().cpu().numpy()
        else:
            outs = []
            for t in range(L):
                obs, rew, done, info = v.step(A[t], auto_reset=False)
                outs.append((obs.cpu().numpy().copy(), rew.cpu().numpy().copy(), done.cpu().numpy().copy(),
                             info.cpu().numpy().copy(), v.assigned_target_ids().cpu().numpy()))
        for e in range(E):
            if ep >= len(eps[e]):
                continue
            for t in range(len(eps[e][ep])):
                o, r, d, inf, asg = outs[t]
                R = res[e]
                R["obs"].append(o[e]); R["reward"].append(r[e]); R["done"].append(int(d[e]))
                R["uav_idx"].append(int(inf[e, _lib.INFO["UAV_IDX"]]))
                R["target_idx"].append(int(inf[e, _lib.INFO["TARGET_IDX"]]))
                R["J_val"].append(inf[e, _lib.INFO["J"]]); R["num_assigned"].append(int(inf[e, 1]))
                R["is_valid"].append(int(inf[e, 2])); R["avg_p_dmg"].append(inf[e, 3])
                R["avg_p_final"].append(inf[e, 4])
                R["assigned"].append(asg[e] if asg is not None else None)
        if fused:
            for e in range(E):
                if ep < len(eps[e]):
                    res[e]["assigned"][-1] = asg_final[e]
        assert int(v.errors().max()) <= 1
    return [{k: np.asarray(x) if k != "assigned" else x for k, x in r.items()} for r in res]


def _groups(traj_npz):
    g = {}
    for c in cases(traj_npz):
        s = sub(traj_npz, c["key"])
        key = (c["N"], c["M"], len(s["nfz_pos"]), len(s["icp_pos"]), tuple(s["params"]))
        g.setdefault(key, []).append(s)
    return g


def test_trajectories_stepwise_vs_reference(traj_npz):
    for key, group in _groups(traj_npz).items():
        got = _replay_batched(group)
        for r, s in zip(got, group):
            r["assigned"] = np.stack(r["assigned"])
            _check_traj(r, s)
            np.testing.assert_allclose(np.stack(r["reset_obs"]), s["reset_obs"], rtol=2e-6, atol=1e-6)


def test_trajectories_fused_vs_stepwise(traj_npz):
    """The T-step fused launch gives the same per-step outputs as T single-step launches."""
    for key, group in list(_groups(traj_npz).items())[:6]:
        a = _replay_batched(group, fused=False)
        b = _replay_batched(group, fused=True)
        for ra, rb, s in zip(a, b, group):
            for k in ("obs", "reward", "done", "uav_idx", "target_idx", "J_val", "num_assigned", "is_valid",
                      "avg_p_dmg", "avg_p_final"):
                np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)
            np.testing.assert_array_equal(ra["assigned"][-1], s["assigned"][-1])


def test_against_oracle_bitwise_decisions(traj_npz):
    """GPU vs CPU oracle on the same injected scene: identical decisions, rewards to 1e-12."""
    import oracle
    s = sub(traj_npz, "c15")  # 16x32
    rng = np.random.default_rng(0)
    v = _venv(1, len(s["uav_load"]), len(s["tgt_value"]), len(s["nfz_pos"]), len(s["icp_pos"]), s["params"])
    v.load_scenes(s)
    env = oracle.OracleEnv(s, s["params"])
    for ep in range(3):
        o_gpu = v.reset(episode=1).cpu().numpy()[0]
        o_cpu = env.reset()
        np.testing.assert_allclose(o_gpu, o_cpu, rtol=1e-6, atol=1e-7)
        done = False
        while not done:
            a = int(rng.random() < 0.4)
            obs_c, r_c, done, info_c = env.step(a)
            obs_g, r_g, d_g, info_g = v.step(torch.tensor([a], dtype=torch.int8, device="cuda"), auto_reset=False)
            assert bool(d_g.item()) == done
            assert abs(r_g.item() - r_c) <= 1e-12 * max(1.0, abs(r_c))
            np.testing.assert_array_equal(info_g.cpu().numpy()[0, [1, 2, 5, 6]], info_c[[1, 2, 5, 6]])
            if not done:
                np.testing.assert_allclose(obs_g.cpu().numpy()[0], obs_c, rtol=1e-6, atol=1e-7)
        np.testing.assert_array_equal(v.assigned_target_ids().cpu().numpy()[0], env.assigned())


def test_auto_reset_state_only(traj_npz):
    """auto_reset: the obs returned with done is the next episode's first window, and the next
    episode replays exactly like a host-driven reset."""
    s = sub(traj_npz, "c1")
    v = _venv(1, len(s["uav_load"]), len(s["tgt_value"]), len(s["nfz_pos"]), len(s["icp_pos"]), s["params"])
    v.load_scenes(s)
    v.reset(episode=1)
    rewards = []
    for i, a in enumerate(s["action"]):
        obs, r, d, info = v.step(torch.tensor([a], dtype=torch.int8, device="cuda"), auto_reset=True)
        rewards.append(r.item())
        if s["done"][i]:
            ep = s["episode"][i]
            if ep + 1 <= s["episode"].max():
                np.testing.assert_allclose(obs.cpu().numpy()[0], s["reset_obs"][ep + 1], rtol=2e-6, atol=1e-6)
            assert int(v.episodes().item()) == ep + 2
    scale = np.maximum(np.abs(s["reward"]), 1e-3)
    assert np.max(np.abs(np.array(rewards) - s["reward"]) / scale) < 1e-9


def test_step_after_done_flags_error(traj_npz):
    s = sub(traj_npz, "c0")
    v = _venv(1, 4, 4, 1, 1, s["params"])
    v.load_scenes(s)
    v.reset(episode=1)
    one = torch.ones(1, dtype=torch.int8, device="cuda")
    for _ in range(4):
        v.step(one, auto_reset=False)
    assert int(v.errors().item()) == 0
    _, r, d, _ = v.step(one, auto_reset=False)
    assert int(v.errors().item()) == 1 and int(d.item()) == 1 and r.item() == 0.0


@pytest.mark.parametrize("N,M,Kn,Ki", [(16, 32, 1, 1), (4, 4, 2, 2), (64, 128, 1, 1), (30, 10, 1, 1)])
def test_scene_generation_properties(N, M, Kn, Ki):
    """On-device Philox scenes follow uav_env.py:65-173's distribution; the pair tables equal the
    CPU oracle's on the generated scene."""
    import oracle
    from uavhip.config import cfg, params_vector
    E = 64
    v = _venv(E, N, M, Kn, Ki, seed=1234)
    v.generate_scenes()
    torch.cuda.synchronize()
    up = v.uav_pos.cpu().numpy(); uv = v.uav_vel.cpu().numpy(); ut = v.uav_type.cpu().numpy()
    assert ((up[..., 0] >= 60) & (up[..., 0] <= 90)).all() and ((up[..., 1] >= 0) & (up[..., 1] <= 160)).all()
    assert ((ut == 2).sum(1) == N // 4).all()
    sp = np.linalg.norm(uv, axis=-1)
    assert np.all(np.where(ut == 1, (sp >= 0.35 - 1e-12) & (sp <= 0.5 + 1e-12), (sp >= 0.75 - 1e-12) & (sp <= 0.9 + 1e-12)))
    cost = v.uav_cost.cpu().numpy()
    np.testing.assert_array_equal(cost, np.where(ut == 1, 1.0, 1.25))
    tv = v.tgt_value.cpu().numpy(); tid = v.tgt_id.cpu().numpy()
    for e in range(E):
        assert sorted(tid[e].tolist()) == list(range(M))
        assert (tv[e] == 4.0).sum() == M // 2 and (tv[e] == 16.0).sum() == 1
    tp = v.tgt_pos.cpu().numpy()
    assert ((tp[..., 0] >= 160) & (tp[..., 0] <= 180)).all()
    assert np.abs(v.tgt_vel.cpu().numpy()).max() <= 0.015
    assert len({tuple(np.round(up[e, 0], 9)) for e in range(E)}) == E  # distinct scenes per env
    prm = params_vector(cfg)
    for e in range(0, E, 16):
        s = dict(uav_pos=up[e], uav_vel=uv[e], uav_load=v.uav_load[e].cpu().numpy(), tgt_pos=tp[e],
                 tgt_vel=v.tgt_vel[e].cpu().numpy(), nfz_pos=v.nfz_pos[e, :Kn].cpu().numpy(),
                 icp_pos=v.icp_pos[e, :Ki].cpu().numpy(), icp_vel=v.icp_vel[e, :Ki].cpu().numpy(), tgt_value=tv[e])
        pd, pp = oracle.score_pairs(s, prm)
        np.testing.assert_allclose(v.p_dmg[e].cpu().numpy(), pd, rtol=RTOL_P, atol=ATOL_P)
        np.testing.assert_allclose(v.p_pen[e].cpu().numpy(), pp, rtol=RTOL_P, atol=ATOL_P)
    # determinism: same seed and episode -> same scene
    w = _venv(E, N, M, Kn, Ki, seed=1234)
    w.generate_scenes()
    assert torch.equal(w.uav_pos, v.uav_pos) and torch.equal(w.p_dmg, v.p_dmg)
    assert (v.istate[:, 8] == 1).all()  # one scene generated per env
    v.generate_scenes()
    assert not torch.equal(w.uav_pos, v.uav_pos)  # the next generation differs


def test_auto_full_reset_regenerates_scene():
    """With full_reset_period P the scene changes exactly when the episode index hits a multiple of
    P: the step kernel flips to the pre-generated spare, whose pair tables match the oracle's, and
    uavhip_scene_refresh regenerates the consumed spare off the step path."""
    import oracle
    from uavhip.config import cfg, params_vector
    v = _venv(8, 4, 4, 1, 1, period=3, seed=7)
    assert v.B == 2
    v.istate[:, 4] = 1
    v.generate_scenes()
    v.reset(episode=1)
    one = torch.ones(8, dtype=torch.int8, device="cuda")
    pos_prev = v.uav_pos.clone()
    for ep in range(2, 8):
        for _ in range(4):  # 4 UAVs x assign = 4 steps per episode
            obs, r, d, _ = v.step(one, auto_reset=True)
        torch.cuda.synchronize()
        assert d.all() and (v.episodes() == ep).all()
        changed = not torch.equal(v.uav_pos, pos_prev)
        assert changed == (ep % 3 == 0), ep
        if changed:
            assert (v.istate[:, 7] == 1).all()  # spare consumed
            s = dict(uav_pos=v.uav_pos[0].cpu().numpy(), uav_vel=v.uav_vel[0].cpu().numpy(),
                     uav_load=v.uav_load[0].cpu().numpy(), tgt_pos=v.tgt_pos[0].cpu().numpy(),
                     tgt_vel=v.tgt_vel[0].cpu().numpy(), nfz_pos=v.nfz_pos[0].cpu().numpy(),
                     icp_pos=v.icp_pos[0].cpu().numpy(), icp_vel=v.icp_vel[0].cpu().numpy(),
                     tgt_value=v.tgt_value[0].cpu().numpy())
            pd, pp = oracle.score_pairs(s, params_vector(cfg))
            np.testing.assert_allclose(v.p_dmg[0].cpu().numpy(), pd, rtol=RTOL_P, atol=ATOL_P)
            # the first window of the new episode is built from the new scene
            assert obs[0, 4, 1].item() == np.float32(v.tgt_value[0, 0].item()) / 16
            v.refresh_scenes()
            torch.cuda.synchronize()
            assert (v.istate[:, 7] == 0).all()
        pos_prev = v.uav_pos.clone()
    assert int(v.errors().max()) == 0


def test_full_reset_without_refresh_flags_error():
    """A second full reset before the spare was refreshed keeps the scene and sets error bit 1."""
    v = _venv(4, 4, 4, 1, 1, period=1, seed=9)
    v.generate_scenes()
    v.reset(episode=1)
    one = torch.ones(4, dtype=torch.int8, device="cuda")
    for _ in range(4):
        v.step(one, auto_reset=True)   # episode 2: flips to the spare
    p1 = v.uav_pos.clone()
    for _ in range(4):
        v.step(one, auto_reset=True)   # episode 3: no fresh spare
    torch.cuda.synchronize()
    assert torch.equal(v.uav_pos, p1) and ((v.errors() & 2) == 2).all()


def test_c5_stress_dims_run():
    """BASELINE config 4 dims (64 UAVs x 128 targets, 2 targets per lane) step cleanly with auto-reset."""
    v = _venv(256, 64, 128, 1, 1, period=200, seed=3)
    v.istate[:, 4] = 1
    v.generate_scenes()
    v.reset(episode=1)
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(50):
        a = (torch.rand(256, device="cuda", generator=g) < 0.3).to(torch.int8)
        obs, r, d, info = v.step(a)
    torch.cuda.synchronize()
    assert torch.isfinite(obs).all() and torch.isfinite(r).all() and (r >= 0).all()
    assert int(v.errors().max()) == 0


@pytest.mark.parametrize("N,M,period", [(16, 32, 3), (8, 16, 2), (4, 4, 5), (32, 32, 0)])
def test_two_envs_per_wave_matches_one_per_wave(N, M, period):
    """Multi-step launches pack two envs into a wave when N, M <= 32 (env_group.hpp). Against the
    one-env-per-wave kernel (checked against the reference above) on the same scenes and actions:
    every output and the whole carried state bitwise, over several launches with auto-reset and
    full resets that flip to refreshed spare scenes."""
    E, T = 4096, 40  # the grouped kernel's minimum batch
    outs = []
    for flags in (4, 5):  # UAVHIP_ENV_NO_REPLAY (| ONE_PER_WAVE): the step-by-step kernels
        v = _venv(E, N, M, 1, 1, period=period, seed=21)
        v.desc.flags = flags
        v.istate[:, 4] = 1
        v.generate_scenes()
        v.reset(episode=1)
        g = torch.Generator(device="cuda").manual_seed(7)
        res = []
        for _ in range(3):
            a = (torch.rand(T, E, device="cuda", generator=g) < 0.6).to(torch.int8)
            obs, r, d, info = v.step(a)
            v.refresh_scenes()
            res += [obs.clone(), r.clone(), d.clone(), info.clone()]
        res += [v.istate.clone(), v.dstate.clone(), v.window.clone(), v.nh_final.clone(), v.nh_pure.clone(),
                v.t_cost.clone(), v.n_lock.clone(), v.assigned.clone()]
        assert int((v.errors() & 1).max()) == 0  # bit 2 (a second full reset before a refresh) may occur
        outs.append(res)
    for x, y in zip(*outs):
        assert torch.equal(x, y)


@pytest.mark.parametrize("N,M,Kn,Ki", [(16, 32, 1, 1), (64, 128, 1, 1), (8, 16, 2, 3), (4, 4, 0, 0), (30, 10, 1, 1)])
def test_score_pairs_tiled_matches_scene_scorer(N, M, Kn, Ki):
    """K1 (one workgroup per env, entity terms staged in LDS) against the per-wave scorer that the
    on-device scene generator runs (the pair math of the reference tests above): bitwise."""
    v = _venv(96, N, M, Kn, Ki, seed=5)
    v.generate_scenes()
    torch.cuda.synchronize()
    want_d, want_p = v._scene["p_dmg"].clone(), v._scene["p_pen"].clone()
    v._scene["p_dmg"].fill_(-1.0)
    v._scene["p_pen"].fill_(-1.0)
    v.score_pairs()
    v.istate[:, 6] ^= 1  # the spare buffer too
    v.score_pairs()
    v.istate[:, 6] ^= 1
    torch.cuda.synchronize()
    assert torch.equal(v._scene["p_dmg"], want_d) and torch.equal(v._scene["p_pen"], want_p)


def _device_scene(v, e):
    keys = ("uav_pos", "uav_vel", "uav_load", "uav_cost", "tgt_pos", "tgt_vel", "tgt_value", "tgt_id", "nfz_pos",
            "icp_pos", "icp_vel")
    s = {k: v.active(k)[e].cpu().numpy() for k in keys}
    s["nfz_pos"] = s["nfz_pos"][:v.Kn]
    s["icp_pos"], s["icp_vel"] = s["icp_pos"][:v.Ki], s["icp_vel"][:v.Ki]
    return s


def test_c5_trajectories_vs_oracle():
    """BASELINE config 4 dims (64 UAVs x 128 targets, two targets per lane) against the CPU oracle
    on the device-generated scenes: one fused 400-step launch per env batch with state-only
    auto-reset; decisions / done / pointer walk / num_assigned / is_valid bit-exact, rewards and J
    to 1e-12, obs to the fp32 bar, and the same launch with fp16 observations (UAVHIP_ENV_OBS_F16)
    emits exactly the fp32 windows rounded to binary16 with every other output bitwise equal."""
    import oracle
    from uavhip import _lib
    E, N, M, T = 6, 64, 128, 400
    outs = {}
    for dt in (torch.float32, torch.float16):
        from uavhip.vec_env import VecUAVEnv
        v = VecUAVEnv(E, N, M, 1, 1, full_reset_period=0, seed=11, obs_dtype=dt)
        v.generate_scenes()
        obs0 = v.reset(episode=1)
        g = torch.Generator(device="cuda").manual_seed(3)
        a = (torch.rand(T, E, device="cuda", generator=g) < 0.35).to(torch.int8)
        obs, r, d, info = v.step(a, auto_reset=True)
        torch.cuda.synchronize()
        outs[dt] = (v, obs0.clone(), a.cpu().numpy(), obs.clone(), r.cpu().numpy(), d.cpu().numpy(),
                    info.cpu().numpy())
    v, obs0, acts, obs, rew, done, info = outs[torch.float32]
    obs_np = obs.cpu().numpy()
    n_done = 0
    for e in range(E):
        env = oracle.OracleEnv(_device_scene(v, e), np.array([v.desc.prm[i] for i in range(_lib.PRM_COUNT)]))
        np.testing.assert_allclose(obs0[e].cpu().numpy(), env.reset(), rtol=2e-6, atol=1e-6)
        for t in range(T):
            o_c, r_c, d_c, i_c = env.step(int(acts[t, e]))
            assert bool(done[t, e]) == d_c, (e, t)
            assert abs(rew[t, e] - r_c) <= 1e-12 * max(1.0, abs(r_c)), (e, t, rew[t, e], r_c)
            np.testing.assert_array_equal(info[t, e, [1, 2, 5, 6]], i_c[[1, 2, 5, 6]])
            assert abs(info[t, e, 0] - i_c[0]) <= 1e-12 * max(1.0, abs(i_c[0]))
            if d_c:
                n_done += 1
                o_c = env.reset()
            np.testing.assert_allclose(obs_np[t, e], o_c, rtol=2e-6, atol=1e-6)
    assert n_done >= E  # every env finished at least one episode inside the launch
    h = outs[torch.float16]
    assert h[3].dtype == torch.float16
    assert torch.equal(h[1], obs0.half()) and torch.equal(h[3], obs.half())
    for i in (2, 4, 5, 6):
        np.testing.assert_array_equal(h[i], outs[torch.float32][i])


def test_fp16_obs_two_envs_per_wave():
    """UAVHIP_ENV_OBS_F16 on the grouped (two envs per wave) multi-step kernel: fp16 obs = fp32 obs
    rounded to binary16, all other outputs bitwise equal."""
    from uavhip.vec_env import VecUAVEnv
    res = []
    for dt in (torch.float32, torch.float16):
        v = VecUAVEnv(4096, 16, 32, 1, 1, full_reset_period=0, seed=4, obs_dtype=dt)
        v.generate_scenes()
        v.reset(episode=1)
        g = torch.Generator(device="cuda").manual_seed(9)
        a = (torch.rand(40, 4096, device="cuda", generator=g) < 0.5).to(torch.int8)
        res.append([x.clone() for x in v.step(a, auto_reset=True)])
    torch.cuda.synchronize()
    assert res[1][0].dtype == torch.float16 and torch.equal(res[1][0], res[0][0].half())
    for x, y in zip(res[0][1:], res[1][1:]):
        assert torch.equal(x, y)


def _replay_twins(E, N, M, period, T, launches, obs_dtype, p_assign, seed, start_done=False):
    """Outputs of `launches` multi-step launches + the whole carried state, for K2r (ONE_PER_WAVE: the
    grouped K2g is not a candidate) and the one-env-per-wave step kernel K2 (NO_REPLAY | ONE_PER_WAVE)
    on twin envs."""
    from uavhip.vec_env import VecUAVEnv
    outs = []
    for flags in (1, 5):
        v = VecUAVEnv(E, N, M, 1, 1, full_reset_period=period, seed=seed, obs_dtype=obs_dtype)
        v.desc.flags |= flags
        v.istate[:, 4] = 1
        v.generate_scenes()
        v.reset(episode=1)
        g = torch.Generator(device="cuda").manual_seed(seed)
        res = []
        if start_done:  # half the envs finished by a launch without auto-reset: K2's error path
            one = torch.ones(E, dtype=torch.int8, device="cuda")
            for _ in range(N):
                v.step(one[None].expand(1, E).contiguous(), auto_reset=False)
            v.reset(mask=(torch.arange(E, device="cuda") % 2 == 0).to(torch.uint8))
        for _ in range(launches):
            a = (torch.rand(T, E, device="cuda", generator=g) < p_assign).to(torch.int8)
            obs, r, d, info = v.step(a)
            v.refresh_scenes()
            res += [obs.clone(), r.clone(), d.clone(), info.clone()]
        res += [v.istate.clone(), v.dstate.clone(), v.window.clone(), v.nh_final.clone(), v.nh_pure.clone(),
                v.t_cost.clone(), v.n_lock.clone(), v.assigned.clone(), v.p_dmg.clone()]
        outs.append(res)
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("E,N,M,period,T,p", [(1024, 8, 16, 3, 200, 0.5), (4096, 16, 32, 2, 100, 0.5),
                                              (300, 4, 4, 5, 131, 0.3), (96, 30, 10, 2, 70, 0.6),
                                              (64, 64, 32, 0, 90, 0.5), (256, 8, 16, 1, 64, 0.9),
                                              (128, 16, 32, 3, 257, 0.05)])
def test_env_replay_matches_sequential_step(E, N, M, period, T, p):
    """K2r (the omega = 0 replay, env_replay.hpp) against K2 (checked against the reference above):
    every output -- windows, rewards, done, info -- and the whole carried state bitwise over three
    launches with auto-reset; full resets flipping to refreshed spares (period 1: a second full reset
    in one launch is refused, error bit 2); chunk boundaries (T not a multiple of the 64- or 32-step
    chunk); skip-heavy and assign-heavy action streams; N up to 64, M up to 32."""
    a, b = _replay_twins(E, N, M, period, T, 3, torch.float32, p, seed=E + N + M)
    assert torch.stack([a[2], a[6], a[10]]).any()  # episodes ended inside the launches
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x, y), i


def test_env_replay_fp16_and_finished_envs():
    """K2r with binary16 observations (BASELINE config 4), and envs that were already finished
    before the launch (auto-reset off earlier): those take K2's error path inside K2r."""
    a, b = _replay_twins(512, 8, 16, 4, 96, 2, torch.float16, 0.5, seed=3, start_done=True)
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x, y), i
    assert int((a[-9][:, 5] & 1).sum()) == 256  # the finished envs flagged the stepping error


def test_env_replay_matches_oracle(traj_npz):
    """K2r directly against the CPU oracle: the golden scenes of one shape, several copies each, a
    random action stream in one 150-step launch with state-only auto-reset, every step replayed
    through oracle.OracleEnv -- done bit-exact, rewards to 1e-12, info to 1e-12, windows to the fp32 bar."""
    import oracle
    from uavhip.vec_env import VecUAVEnv
    groups = {}
    for c in cases(traj_npz):
        s = sub(traj_npz, c["key"])
        if s["params"][6] == 0.0 and len(s["nfz_pos"]) == 1:
            groups.setdefault((c["N"], c["M"]), []).append(s)
    (N, M), scenes = max(((k, g) for k, g in groups.items() if k[1] <= 32), key=lambda kv: kv[0][0] * kv[0][1])
    scenes = (scenes * 8)[:32]
    E, T = len(scenes), 150
    v = VecUAVEnv(E, N, M, 1, 1, full_reset_period=0)
    v.set_params(scenes[0]["params"])
    v.load_scenes(scenes)
    v.reset(episode=1)
    rng = np.random.default_rng(5)
    acts = (rng.random((T, E)) < 0.5).astype(np.int8)
    obs, rew, done, info = (x.cpu().numpy() for x in v.step(torch.from_numpy(acts).cuda()))
    refs = [oracle.OracleEnv(s, s["params"]) for s in scenes]
    for r in refs:
        r.reset()
    for t in range(T):
        for e in range(E):
            o_c, r_c, d_c, inf_c = refs[e].step(int(acts[t, e]))
            assert bool(done[t, e]) == d_c, (t, e)
            assert abs(rew[t, e] - r_c) <= 1e-12 * max(1.0, abs(r_c)), (t, e)
            np.testing.assert_allclose(info[t, e, :5], inf_c[:5], rtol=1e-12, atol=1e-15)
            np.testing.assert_array_equal(info[t, e, 5:7], inf_c[5:7])
            if d_c:
                o_c = refs[e].reset()
            np.testing.assert_allclose(obs[t, e], o_c, rtol=2e-6, atol=1e-6)
    assert done.any()


def test_negative_values_disable_the_replay_kernel(traj_npz):
    """K2r needs every assign accepted (omega = 0 AND target values >= 0). A host scene with a
    negative target value makes VecUAVEnv.load_scenes set UAVHIP_ENV_NO_REPLAY, so a 120-step launch
    takes the step-by-step kernel and matches the CPU oracle (whose reject branch, uav_env.py:317-338,
    fires on the negative-value target) -- decisions bit-exact, rewards to 1e-12."""
    import oracle
    from uavhip import _lib
    from uavhip.vec_env import VecUAVEnv
    s = None
    for c in cases(traj_npz):
        cand = sub(traj_npz, c["key"])
        if cand["params"][6] == 0.0 and c["M"] <= 32 and len(cand["nfz_pos"]) == 1:
            s = cand
            break
    s = dict(s)
    s["tgt_value"] = np.asarray(s["tgt_value"], np.float64).copy()
    s["tgt_value"][::2] *= -1.0  # every other target a liability
    E, T = 16, 120
    v = VecUAVEnv(E, int(len(s["uav_load"])), int(len(s["tgt_value"])), 1, 1, full_reset_period=0)
    v.set_params(s["params"])
    assert not v.desc.flags & _lib.ENV_NO_REPLAY
    v.load_scenes([s] * E)
    assert v.desc.flags & _lib.ENV_NO_REPLAY
    v.reset(episode=1)
    acts = (np.random.default_rng(2).random((T, E)) < 0.6).astype(np.int8)
    obs, rew, done, info = (x.cpu().numpy() for x in v.step(torch.from_numpy(acts).cuda()))
    refs = [oracle.OracleEnv(s, s["params"]) for _ in range(E)]
    for r in refs:
        r.reset()
    rejects = 0
    for t in range(T):
        for e in range(E):
            o_c, r_c, d_c, inf_c = refs[e].step(int(acts[t, e]))
            rejects += int(acts[t, e] == 1 and inf_c[2] == 0)
            assert bool(done[t, e]) == d_c, (t, e)
            assert abs(rew[t, e] - r_c) <= 1e-12 * max(1.0, abs(r_c)), (t, e)
            np.testing.assert_array_equal(info[t, e, 5:7], inf_c[5:7])
            if d_c:
                refs[e].reset()
    print(f"rejected assigns: {rejects}")
    assert rejects > 0


def test_configs4_shard_at_size():
    """BASELINE configs[4]'s per-GPU shard at its own size: 8192 envs x 64 UAVs x 128 targets, fp16
    observations, auto-reset with full_reset_period 200 (main_train.py:79), 200 steps.
    (1) One 200-step launch (K2 one env per wave: M > 32 rules out the grouped and replay kernels)
        against 200 single-step launches of twin envs: every output and the carried state bitwise.
    (2) Every env: rewards / info finite, no stepping errors, >= 95 % of them ended an episode, and the fp16 windows
        are exactly the fp32 run's windows rounded to binary16 (twin envs, f32 observations).
    (3) 8 sampled envs replayed through the CPU oracle on their device-generated scenes: done /
        pointer / num_assigned / is_valid bit-exact, rewards and J to 1e-12 (uav_env.py:295-435)."""
    import oracle
    from uavhip import _lib
    from uavhip.vec_env import VecUAVEnv
    E, N, M, T = 8192, 64, 128, 200
    g = torch.Generator(device="cuda").manual_seed(12)
    acts = (torch.rand(T, E, device="cuda", generator=g) < 0.4).to(torch.int8)

    def make(dt):
        v = VecUAVEnv(E, N, M, 1, 1, full_reset_period=200, seed=13, obs_dtype=dt)
        v.istate[:, _lib.IST["EPISODE"]] = 1
        v.generate_scenes()
        return v, v.reset(episode=1).clone()

    v16, obs0_16 = make(torch.float16)
    obs16, r16, d16, i16 = (x.clone() for x in v16.step(acts))
    state16 = [x.clone() for x in (v16.istate, v16.dstate, v16.window, v16.nh_final, v16.assigned)]
    # (1) the same 200 steps as single-step launches
    w16, _ = make(torch.float16)
    singles = [[x.clone() for x in w16.step(acts[t])] for t in range(T)]
    for k, name in enumerate(("obs", "reward", "done", "info")):
        assert torch.equal(torch.stack([s[k] for s in singles]), (obs16, r16, d16, i16)[k]), name
    for a, b in zip(state16, (w16.istate, w16.dstate, w16.window, w16.nh_final, w16.assigned)):
        assert torch.equal(a, b)
    del singles, w16
    # (2) properties of every env + the fp16 windows against the fp32 twin's
    assert torch.isfinite(r16).all() and torch.isfinite(i16).all() and (r16 >= 0).all()
    assert int(v16.errors().max()) == 0
    ends = d16.sum(0)
    assert int((ends > 0).sum()) >= 0.95 * E  # an episode is ~160 steps at 64 x 128 (p_assign 0.4)
    v32, obs0_32 = make(torch.float32)
    obs32, r32, d32, i32 = (x.clone() for x in v32.step(acts))
    assert torch.equal(obs0_16, obs0_32.half()) and torch.equal(obs16, obs32.half())
    assert torch.equal(r16, r32) and torch.equal(d16, d32) and torch.equal(i16, i32)
    # (3) 8 envs through the CPU oracle
    rew, done, info, a_np = r32.cpu().numpy(), d32.cpu().numpy(), i32.cpu().numpy(), acts.cpu().numpy()
    prm = np.array([v32.desc.prm[i] for i in range(_lib.PRM_COUNT)])
    fresh, _ = make(torch.float32)  # the scenes before any reset (no full reset within 200 steps)
    for e in np.random.default_rng(1).choice(E, 8, replace=False):
        ref = oracle.OracleEnv(_device_scene(fresh, int(e)), prm)
        ref.reset()
        for t in range(T):
            o_c, r_c, d_c, i_c = ref.step(int(a_np[t, e]))
            assert bool(done[t, e]) == d_c, (e, t)
            assert abs(rew[t, e] - r_c) <= 1e-12 * max(1.0, abs(r_c)), (e, t, rew[t, e], r_c)
            np.testing.assert_array_equal(info[t, e, [1, 2, 5, 6]], i_c[[1, 2, 5, 6]])
            assert abs(info[t, e, 0] - i_c[0]) <= 1e-12 * max(1.0, abs(i_c[0]))
            if d_c:
                ref.reset()
    print(f"configs[4] shard: {int(ends.sum())} episodes ended over {E} envs x {T} steps")


def test_configs1_k2r_at_size_vs_oracle():
    """BASELINE configs[1] at its own size: 1024 envs x 8 UAVs x 16 targets, one 256-step env-only
    launch (K2r, the omega = 0 replay: auto-reset, full_reset_period 200 as main_train.py:79) on
    device-generated scenes; 8 sampled envs replayed step by step through the CPU oracle
    (uav_env.py:295-435) -- done / num_assigned / is_valid bit-exact, rewards and J to 1e-12,
    windows to the fp32 bar (2e-6) -- and every env's outputs finite with no stepping error."""
    import oracle
    from uavhip import _lib
    from uavhip.vec_env import VecUAVEnv
    E, N, M, T = 1024, 8, 16, 256
    v = VecUAVEnv(E, N, M, 1, 1, full_reset_period=200, seed=21)
    v.istate[:, _lib.IST["EPISODE"]] = 1
    v.generate_scenes()
    scenes = {}
    picks = [int(e) for e in np.random.default_rng(4).choice(E, 8, replace=False)]
    for e in picks:
        scenes[e] = _device_scene(v, e)
    obs0 = v.reset(episode=1).cpu().numpy()
    g = torch.Generator(device="cuda").manual_seed(22)
    acts = (torch.rand(T, E, device="cuda", generator=g) < 0.5).to(torch.int8)
    obs, rew, done, info = (x.cpu().numpy() for x in v.step(acts))
    assert np.isfinite(rew).all() and np.isfinite(info).all() and int(v.errors().max()) == 0
    prm = np.array([v.desc.prm[i] for i in range(_lib.PRM_COUNT)])
    a_np = acts.cpu().numpy()
    ends = 0
    for e in picks:
        ref = oracle.OracleEnv(scenes[e], prm)
        np.testing.assert_allclose(obs0[e], ref.reset(), rtol=2e-6, atol=1e-6)
        for t in range(T):
            o_c, r_c, d_c, i_c = ref.step(int(a_np[t, e]))
            assert bool(done[t, e]) == d_c, (e, t)
            assert abs(rew[t, e] - r_c) <= 1e-12 * max(1.0, abs(r_c)), (e, t, rew[t, e], r_c)
            np.testing.assert_array_equal(info[t, e, [1, 2, 5, 6]], i_c[[1, 2, 5, 6]])
            assert abs(info[t, e, 0] - i_c[0]) <= 1e-12 * max(1.0, abs(i_c[0]))
            if d_c:
                ends += 1
                o_c = ref.reset()
            np.testing.assert_allclose(obs[t, e], o_c, rtol=2e-6, atol=1e-6)
    print(f"configs[1]: {ends} episodes ended in the 8 replayed envs; {int(done.sum())} over all {E} envs")
    assert ends > 8


def test_configs2_rollout_iteration_at_size_vs_oracle():
    """BASELINE configs[2] at its own size: one full k_rollout_steps iteration over 4096 envs x 16
    UAVs x 32 targets, T = 64 (window-row forward + sampling + env step, auto-reset, full_reset_period
    200) on device-generated scenes. 8 sampled envs replayed through the CPU oracle with the actions
    the kernel sampled -- done bit-exact, rewards and J to 1e-12, windows to 2e-6 -- and their
    log-probabilities / values against the torch fp32 `evaluate` of the same windows and actions
    (transformer_net.py:124-144; 1e-5). Every env's outputs finite."""
    import oracle
    from uavhip import _lib
    from uavhip.policy import TransformerActorCritic
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv
    E, N, M, T = 4096, 16, 32, 64
    torch.manual_seed(23)
    pol = TransformerActorCritic().cuda()
    v = VecUAVEnv(E, N, M, 1, 1, full_reset_period=200, seed=24)
    eng = RolloutEngine(v, pol, T, seed=25)
    assert eng.persistent
    eng.start()
    picks = [int(e) for e in np.random.default_rng(6).choice(E, 8, replace=False)]
    scenes = {e: _device_scene(v, e) for e in picks}
    tr = eng.collect()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.logp).all() and torch.isfinite(tr.values).all() and torch.isfinite(tr.rewards).all()
    assert int((v.errors() & 1).max()) == 0
    prm = np.array([v.desc.prm[i] for i in range(_lib.PRM_COUNT)])
    obs, act = tr.obs.cpu().numpy(), tr.actions.cpu().numpy()
    rew, done, info = tr.rewards.cpu().numpy(), tr.dones.cpu().numpy(), tr.info.cpu().numpy()
    ends = 0
    for e in picks:
        ref = oracle.OracleEnv(scenes[e], prm)
        np.testing.assert_allclose(obs[0, e], ref.reset(), rtol=2e-6, atol=1e-6)
        for t in range(T):
            o_c, r_c, d_c, i_c = ref.step(int(act[t, e]))
            assert bool(done[t, e]) == d_c, (e, t)
            assert abs(rew[t, e] - r_c) <= 1e-12 * max(1.0, abs(r_c)), (e, t, rew[t, e], r_c)
            np.testing.assert_array_equal(info[t, e, [1, 2, 5, 6]], i_c[[1, 2, 5, 6]])
            assert abs(info[t, e, 0] - i_c[0]) <= 1e-12 * max(1.0, abs(i_c[0]))
            if d_c:
                ends += 1
                o_c = ref.reset()
            np.testing.assert_allclose(obs[t + 1, e], o_c, rtol=2e-6, atol=1e-6)
    idx = torch.tensor(picks, device="cuda")
    x = tr.obs[:T, idx].reshape(T * len(picks), 5, 14)
    a = tr.actions[:, idx].reshape(-1).long()
    with torch.no_grad():
        lp_t, v_t, _ = pol.evaluate(x, a)
    torch.testing.assert_close(tr.logp[:, idx].reshape(-1), lp_t, rtol=1e-5, atol=2e-6)
    torch.testing.assert_close(tr.values[:, idx].reshape(-1), v_t[:, 0], rtol=1e-5, atol=1e-5)
    print(f"configs[2]: {ends} episodes ended in the 8 replayed envs over {T} steps")
