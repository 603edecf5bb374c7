"""GPU parity of the fused policy forward (policy.hip) and the GAE kernels (gae.hip), plus the
drop-in UAVEnv / PPOAgent and the batched rollout engine. Marked gpu.

Policy tolerance (fp32 vs fp32 in a different summation order, transformer depth 2): logits /
logp / entropy 2e-6 absolute + 1e-5 relative, value 1e-5 absolute + 1e-5 relative -- measured on
MI355X (the tests print them): at most 7e-7 absolute on logits / logp / entropy and 2.4e-6 on
values of magnitude ~10, i.e. 1e-5 relative is the north_star bar with a 3-10x margin. GAE returns
bit-exact."""
import random

import numpy as np
import pytest
import torch

from conftest import assert_close_report, cases, has_gpu, sub

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]


def _load_policy(policy_npz, tag):
    from uavhip.policy import TransformerActorCritic
    net = TransformerActorCritic()
    sd = {k[len(f"{tag}/w/"):]: torch.from_numpy(policy_npz[k].copy()) for k in policy_npz.files
          if k.startswith(f"{tag}/w/")}
    net.load_state_dict(sd)
    return net.cuda()


@pytest.mark.parametrize("tag", ["a", "b"])
def test_row_projection_forward_vs_reference(policy_npz, tag):
    """uavhip_policy_forward_rows with fill (every window's rows projected afresh) against the
    reference's outputs on the golden windows, at the full-forward tolerance."""
    from uavhip.policy import rowproj_buffer
    net = _load_policy(policy_npz, tag)
    x = torch.from_numpy(policy_npz["states"]).cuda()
    a = torch.from_numpy(policy_npz["actions"]).cuda()
    B = x.shape[0]
    ent = torch.empty(B, device="cuda")
    lg = torch.empty(B, 2, device="cuda")
    _, logp, value, ent, lg = net.fused_forward(x, actions=a, entropy=ent, logits=lg, rowproj=rowproj_buffer(B),
                                                step=3, fill=True)
    torch.cuda.synchronize()
    assert_close_report(f"{tag} logits", lg.cpu().numpy(), policy_npz[f"{tag}/logits"], rtol=1e-5, atol=2e-6)
    assert_close_report(f"{tag} logp", logp.cpu().numpy(), policy_npz[f"{tag}/logp"], rtol=1e-5, atol=2e-6)
    assert_close_report(f"{tag} entropy", ent.cpu().numpy(), policy_npz[f"{tag}/entropy"], rtol=1e-5, atol=2e-6)
    assert_close_report(f"{tag} value", value.cpu().numpy(), policy_npz[f"{tag}/value"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B,step0", [(200, 0), (4096, 7)])
def test_row_projection_sequence(B, step0):
    """A deque window sequence (oracle.windows restatement: shifts, episode ends -> zero padding)
    through the ring: each step projects only its new row. Bitwise equal to rebuilding every
    window's rows at every step (fill), and within fp32 rounding of the full forward."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle.windows import windows_from_rows
    from uavhip.policy import TransformerActorCritic, rowproj_buffer
    torch.manual_seed(2)
    net = TransformerActorCritic().cuda()
    T = 12
    g = np.random.default_rng(B)
    first = g.standard_normal((B, 5, 14)).astype(np.float32)
    first[: B // 3, :3] = 0
    first[B // 3: B // 2, :4] = 0
    rows = g.standard_normal((T, B, 14)).astype(np.float32)
    dones = g.random((T, B)) < 0.15
    wins = torch.from_numpy(windows_from_rows(first, rows, dones)).cuda()
    acts = torch.from_numpy((g.random((T, B)) < 0.5).astype(np.int8)).cuda()
    ring, fresh = rowproj_buffer(B), rowproj_buffer(B)
    for t in range(T):
        outs = []
        for buf, fill in ((ring, t == 0), (fresh, True), (None, False)):
            lg = torch.empty(B, 2, device="cuda")
            kw = dict(rowproj=buf, step=step0 + t, fill=fill) if buf is not None else {}
            _, lp, v, _, lg = net.fused_forward(wins[t], actions=acts[t], logits=lg, **kw)
            outs.append((lg, lp, v))
        torch.cuda.synchronize()
        for x, y in zip(outs[0], outs[1]):
            assert torch.equal(x, y), f"step {t}: ring != fill"
        for x, y in zip(outs[0], outs[2]):
            torch.testing.assert_close(x, y, rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("B", [200, 4096])
def test_value_rows_matches_forward_rows(B):
    """uavhip_policy_value_rows (the rollout's bootstrap: critic trunk + head only) against the full
    ring forward's value, bitwise, along a window sequence whose steps advance the ring through the
    full forward -- with fill, and on the ring the previous steps left (fill = 0)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle.windows import windows_from_rows
    from uavhip.policy import TransformerActorCritic, rowproj_buffer
    torch.manual_seed(3)
    net = TransformerActorCritic().cuda()
    T = 6
    g = np.random.default_rng(B + 1)
    first = g.standard_normal((B, 5, 14)).astype(np.float32)
    first[: B // 4, :2] = 0
    rows = g.standard_normal((T, B, 14)).astype(np.float32)
    dones = g.random((T, B)) < 0.2
    wins = torch.from_numpy(windows_from_rows(first, rows, dones)).cuda()
    ring, fresh = rowproj_buffer(B), rowproj_buffer(B)
    for t in range(T):
        before = ring.clone()  # the ring the full forward of steps 0 .. t-1 left
        _, _, v, _, _ = net.fused_forward(wins[t], rowproj=ring, step=t, fill=t == 0)
        v_fill = net.value_rows(wins[t], fresh, t, torch.empty(B, device="cuda"), fill=True)
        torch.cuda.synchronize()
        assert torch.equal(v, v_fill), f"step {t}: value_rows(fill) != forward_rows value"
        if t > 0:
            v_ring = net.value_rows(wins[t], before, t, torch.empty(B, device="cuda"))
            torch.cuda.synchronize()
            assert torch.equal(v, v_ring), f"step {t}: value_rows(ring) != forward_rows value"


@pytest.mark.parametrize("tag", ["a", "b"])
def test_fused_policy_vs_reference(policy_npz, tag):
    net = _load_policy(policy_npz, tag)
    x = torch.from_numpy(policy_npz["states"]).cuda()
    a = torch.from_numpy(policy_npz["actions"]).cuda()
    B = x.shape[0]
    ent = torch.empty(B, device="cuda")
    lg = torch.empty(B, 2, device="cuda")
    _, logp, value, ent, lg = net.fused_forward(x, actions=a, entropy=ent, logits=lg)
    torch.cuda.synchronize()
    assert_close_report(f"{tag} logits", lg.cpu().numpy(), policy_npz[f"{tag}/logits"], rtol=1e-5, atol=2e-6)
    assert_close_report(f"{tag} logp", logp.cpu().numpy(), policy_npz[f"{tag}/logp"], rtol=1e-5, atol=2e-6)
    assert_close_report(f"{tag} entropy", ent.cpu().numpy(), policy_npz[f"{tag}/entropy"], rtol=1e-5, atol=2e-6)
    assert_close_report(f"{tag} value", value.cpu().numpy(), policy_npz[f"{tag}/value"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B", [1, 7, 16, 300, 4096])
def test_fused_policy_vs_torch_module(policy_npz, B):
    """Random windows with every padding pattern, batch tails (B % 16 != 0) and the C3 batch."""
    net = _load_policy(policy_npz, "b")
    g = torch.Generator().manual_seed(B)
    x = torch.randn(B, 5, 14, generator=g) * 0.7
    pad = torch.randint(0, 5, (B,), generator=g)
    for i in range(B):
        x[i, :pad[i]] = 0.0
    x = x.cuda()
    a = torch.randint(0, 2, (B,), generator=g).cuda()
    with torch.no_grad():
        logp_t, v_t, ent_t = net.evaluate(x, a)
    ent = torch.empty(B, device="cuda")
    _, logp, value, ent, _ = net.fused_forward(x, actions=a, entropy=ent)
    assert_close_report(f"B={B} logp", logp.cpu().numpy(), logp_t.cpu().numpy(), rtol=1e-5, atol=2e-6)
    assert_close_report(f"B={B} entropy", ent.cpu().numpy(), ent_t.cpu().numpy(), rtol=1e-5, atol=2e-6)
    assert_close_report(f"B={B} value", value.cpu().numpy(), v_t[:, 0].cpu().numpy(), rtol=1e-5, atol=1e-5)


def test_fused_sampling_distribution(policy_npz):
    net = _load_policy(policy_npz, "a")
    x = torch.from_numpy(np.repeat(policy_npz["states"][:1], 65536, axis=0)).cuda()
    lg = torch.empty(65536, 2, device="cuda")
    act, logp, _, _, lg = net.fused_forward(x, logits=lg, seed=99, offset=0)
    p1 = torch.softmax(lg[0], -1)[1].item()
    freq = act.float().mean().item()
    assert abs(freq - p1) < 5 * np.sqrt(p1 * (1 - p1) / 65536) + 1e-4
    lp_expected = torch.log_softmax(lg, -1).gather(1, act.long()[:, None])[:, 0]
    torch.testing.assert_close(logp, lp_expected, rtol=1e-5, atol=1e-6)


def test_gae_vs_reference(gae_npz):
    from uavhip.ppo import gae
    for c in cases(gae_npz):
        s = sub(gae_npz, c["key"])
        ret, adv, stats = gae(torch.from_numpy(s["rewards"]), torch.from_numpy(s["dones"]),
                              torch.from_numpy(s["values"]).cuda())
        np.testing.assert_array_equal(ret.cpu().numpy(), s["returns"])  # bit-exact fp32 recurrence
        np.testing.assert_allclose(adv.cpu().numpy(), s["advantages"], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("T,E,boot", [(64, 4096, True), (7, 33, False), (1, 5, True), (300, 64, True)])
def test_gae_2d_vs_oracle(T, E, boot):
    from oracle import gae as ogae
    from uavhip.ppo import gae
    rng = np.random.default_rng(T * 1000 + E)
    r = np.where(rng.random((T, E)) < 0.5, 0.0, rng.uniform(0, 3, (T, E)))
    d = (rng.random((T, E)) < 0.05).astype(np.uint8)
    v = rng.normal(size=(T, E)).astype(np.float32) * 3
    lv = rng.normal(size=E).astype(np.float32) if boot else None
    ret, adv, stats = gae(torch.from_numpy(r), torch.from_numpy(d), torch.from_numpy(v).cuda(),
                          None if lv is None else torch.from_numpy(lv).cuda(), normalize=False)
    r_o, a_o = ogae.gae_2d(r, d, v, last_values=lv)
    np.testing.assert_array_equal(ret.cpu().numpy(), r_o)
    np.testing.assert_array_equal(adv.cpu().numpy(), a_o)
    ret2, adv2, stats = gae(torch.from_numpy(r), torch.from_numpy(d), torch.from_numpy(v).cuda(),
                            None if lv is None else torch.from_numpy(lv).cuda())
    if T * E > 1:
        a_n, mean, std = ogae.normalize(a_o)
        np.testing.assert_allclose(adv2.cpu().numpy(), a_n, rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(stats.cpu().numpy(), [mean, std], rtol=1e-6)


def test_dropin_uavenv_reproduces_reference(traj_npz):
    """envs.uav_env.UAVEnv seeded like the reference replays the reference's trajectories:
    same scenes from the global numpy/random streams, same per-step outputs."""
    from uavhip.config import cfg, config0_overrides
    from envs.uav_env import UAVEnv
    saved = {k: getattr(cfg, k) for k in ("NUM_UAVS", "NUM_TARGETS", "COST_WEIGHT_OMEGA")}
    try:
        for c in cases(traj_npz)[:24]:
            if c["cfg"] != "A":
                continue
            s = sub(traj_npz, c["key"])
            cfg.NUM_UAVS, cfg.NUM_TARGETS, cfg.COST_WEIGHT_OMEGA = c["N"], c["M"], c["omega"]
            np.random.seed(c["seed"]); random.seed(c["seed"])
            env = UAVEnv()
            ep = -1
            for i, a in enumerate(s["action"]):
                if s["episode"][i] != ep:
                    ep = s["episode"][i]
                    o = env.reset(full_reset=(ep == 0))
                    np.testing.assert_allclose(o, s["reset_obs"][ep], rtol=2e-6, atol=1e-6)
                    if ep == 0:
                        np.testing.assert_array_equal([t.id for t in env.targets], s["tgt_id"])
                obs, r, d, info = env.step(int(a))
                assert d == bool(s["done"][i])
                assert abs(r - s["reward"][i]) <= 1e-9 * max(1e-3, abs(s["reward"][i]))
                assert info["num_assigned"] == s["num_assigned"][i]
                iv = s["is_valid"][i]
                assert info["is_valid_action"] == (None if iv < 0 else bool(iv))
                assert env.uav_idx == s["uav_idx"][i] and env.target_idx == s["target_idx"][i]
                if d:
                    assert obs.shape == (14,) and not obs.any()
                else:
                    np.testing.assert_allclose(obs, s["obs"][i], rtol=2e-6, atol=1e-6)
            np.testing.assert_array_equal([u.assigned_target_id for u in env.uavs], s["assigned"][-1])
            with pytest.raises(IndexError):
                env.step(0)
    finally:
        for k, v in saved.items():
            setattr(cfg, k, v)
    del config0_overrides


def test_dropin_ppoagent_loop():
    """main_train.py:79-146 shape of use: select_action / store_transition / update."""
    from envs.uav_env import UAVEnv
    from agents.ppo import PPOAgent
    from uavhip.config import cfg
    saved = (cfg.NUM_UAVS, cfg.NUM_TARGETS)
    try:
        cfg.NUM_UAVS, cfg.NUM_TARGETS = 8, 8
        np.random.seed(0); random.seed(0); torch.manual_seed(0)
        env, agent = UAVEnv(), PPOAgent()
        for ep in range(1, 30):
            state = env.reset(full_reset=(ep == 1))
            done = False
            while not done:
                a = agent.select_action(state)
                state, r, done, info = env.step(a)
                agent.store_transition(r, done)
            if len(agent.buffer["states"]) >= 64:
                stats = agent.update()
                assert stats is not None and all(np.isfinite(list(stats.values())))
                assert len(agent.buffer["states"]) == 0
                break
        else:
            pytest.fail("no update happened")
        # policy_old got the new weights and the fused path picked them up
        x = torch.zeros(1, 5, 14, device="cuda"); x[0, -1, 0] = 0.5
        a1 = agent.policy_old.fused_forward(x, actions=torch.zeros(1, dtype=torch.long, device="cuda"))[1]
        lp, _, _ = agent.policy.evaluate(x, torch.zeros(1, dtype=torch.long, device="cuda"))
        torch.testing.assert_close(a1, lp.detach(), rtol=1e-5, atol=2e-6)
    finally:
        cfg.NUM_UAVS, cfg.NUM_TARGETS = saved


def test_rollout_engine_invariants():
    from uavhip import _lib
    from uavhip.policy import TransformerActorCritic
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv
    torch.manual_seed(0)
    E, T = 512, 40
    env = VecUAVEnv(E, 16, 32, 1, 1, seed=5)
    pol = TransformerActorCritic().cuda()
    eng = RolloutEngine(env, pol, T, seed=11)
    eng.start()
    tr = eng.collect()
    torch.cuda.synchronize()
    d = tr.dones.cpu().numpy().astype(bool)
    r = tr.rewards.cpu().numpy()
    assert d.any() and (r >= 0).all() and np.isfinite(r).all()
    obs_next = tr.obs[1:].cpu().numpy()
    # after a done the next window is a fresh episode: 4 zero rows then the first feature row
    assert (obs_next[d][:, :4] == 0).all() and (obs_next[d][:, 4, 13] == 1.0).all()
    info = tr.info.cpu().numpy()
    assert (info[..., _lib.INFO["IS_VALID"]][tr.actions.cpu().numpy() == 0] == -1).all()
    ret, adv = tr.ret.cpu().numpy(), tr.adv.cpu().numpy()
    assert np.isfinite(ret).all() and abs(adv.mean()) < 1e-4 and abs(adv.std(ddof=1) - 1) < 1e-3
    eng.roll()
    eng.collect()
    assert int(env.errors().max()) == 0


def test_compact_exchange_rebuilds_rollout_windows():
    """The data-parallel exchange format (uavhip/dist.py): a real rollout's windows come back
    bit-exactly from the rows / done flags / first windows (uavhip_windows_from_rows), for several
    iterations (windows carried across the iteration boundary) and several payload blocks, and the
    GPU rebuild equals the oracle's step-by-step deque restatement on random inputs."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle.windows import windows_from_rows
    from uavhip import dist as udist
    from uavhip.policy import TransformerActorCritic
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv
    torch.manual_seed(0)
    E, T = 192, 24
    env = VecUAVEnv(E, 4, 6, 1, 1, seed=9)  # short episodes: many boundaries inside a window
    eng = RolloutEngine(env, TransformerActorCritic().cuda(), T, seed=3)
    eng.start()
    pays, wins = [], []
    for _ in range(3):
        tr = eng.collect()
        assert tr.dones.any()
        pays.append(udist.pack_compact(tr.obs, tr.actions, tr.logp, tr.values, tr.ret, tr.adv, tr.dones))
        wins.append(tr.obs[:T].clone())
    got = udist.unpack_compact(torch.stack(pays), T, E)
    torch.cuda.synchronize()
    assert torch.equal(got["obs"], torch.cat(wins).reshape(-1, 5, 14))
    assert torch.equal(got["dones"].reshape(3, T, E).to(torch.uint8).cpu(), torch.stack(
        [udist_p[T * E * 14:T * E * 20].reshape(T, E, 6)[..., 5].cpu().to(torch.uint8) for udist_p in pays]))
    # random inputs against the oracle (zero rows included)
    g = torch.Generator().manual_seed(4)
    first = torch.randn(2, E, 5, 14, generator=g)
    rows = torch.randn(2, T, E, 14, generator=g)
    dn = (torch.rand(2, T, E, generator=g) < 0.3)
    pay = torch.stack([torch.cat([rows[b].reshape(-1), torch.stack([torch.zeros(T, E)] * 5 + [dn[b].float()], -1)
                                  .reshape(-1), first[b].reshape(-1)]) for b in range(2)]).cuda()
    got = udist.unpack_compact(pay, T, E)["obs"].reshape(2, T, E, 5, 14).cpu().numpy()
    for b in range(2):
        np.testing.assert_array_equal(got[b], windows_from_rows(first[b].numpy(), rows[b].numpy(), dn[b].numpy()))


def test_rollout_row_cache_matches_full_forward():
    """The rollout's window-row path (every step after t = 0 projects one row) against the
    full-window forward on the recorded windows and actions: logp / value within fp32 rounding."""
    from uavhip.policy import TransformerActorCritic
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv
    torch.manual_seed(0)
    E, T = 256, 24
    env = VecUAVEnv(E, 4, 6, 1, 1, seed=9)
    pol = TransformerActorCritic().cuda()
    eng = RolloutEngine(env, pol, T, seed=3)
    eng.start()
    for _ in range(2):
        tr = eng.collect()
        assert tr.dones.any()
        x = tr.obs[:T].reshape(-1, 5, 14)
        _, lp, v, _, _ = pol.fused_forward(x, actions=tr.actions.reshape(-1))
        torch.cuda.synchronize()
        torch.testing.assert_close(lp, tr.logp.reshape(-1), rtol=1e-5, atol=2e-6)
        torch.testing.assert_close(v, tr.values.reshape(-1), rtol=1e-5, atol=2e-6)


def test_rollout_graph_replay_matches_eager():
    """The captured hipGraph iteration reproduces eager launches bit for bit (same device state,
    same sampling counters), across several replays and a weight change in between."""
    from uavhip.policy import TransformerActorCritic
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv
    outs = []
    for graph in (False, True):
        torch.manual_seed(0)
        env = VecUAVEnv(256, 8, 16, 1, 1, seed=3, full_reset_period=2)
        pol = TransformerActorCritic().cuda()
        eng = RolloutEngine(env, pol, 16, seed=4)
        eng.start()
        if graph:
            eng.capture()
            eng.counter.zero_()
            # capture ran the body once on a side stream: rewind the device state
            env2 = VecUAVEnv(256, 8, 16, 1, 1, seed=3, full_reset_period=2)
            env2.istate[:, 4] = 1
            env2.generate_scenes()
            for name in ("nh_final", "nh_pure", "t_cost", "n_lock", "assigned", "istate", "dstate", "window"):
                getattr(env, name).copy_(getattr(env2, name))
            for k in env._scene:
                env._scene[k].copy_(env2._scene[k])
            env.reset(episode=1, obs_out=eng.traj.obs[eng.T])
        res = []
        for it in range(4):
            if it == 2:
                with torch.no_grad():
                    pol.actor_head[2].bias.add_(0.5)   # weights change between iterations
            tr = eng.collect()
            torch.cuda.synchronize()
            res.append([x.clone() for x in (tr.actions, tr.rewards, tr.dones, tr.obs, tr.adv, tr.values)])
        outs.append(res)
    for a, b in zip(*outs):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


def test_graph_ppo_update_matches_eager():
    """GraphPPOUpdater replays == ppo_epochs eager steps (same minibatch order, same Adam)."""
    import copy
    from uavhip.policy import TransformerActorCritic
    from uavhip.ppo import GraphPPOUpdater, make_optimizer, ppo_epochs
    torch.manual_seed(3)
    base = TransformerActorCritic().cuda()
    n, bs = 1024, 256
    g = torch.Generator(device="cpu").manual_seed(11)
    states = torch.randn(n, 5, 14, generator=g).cuda()
    states[: n // 4, :2] = 0
    acts = torch.randint(0, 2, (n,), generator=g).cuda()
    logp = -torch.rand(n, generator=g).cuda()
    vals, ret, adv = (torch.randn(n, generator=g).cuda() for _ in range(3))
    pe, pg = copy.deepcopy(base), copy.deepcopy(base)
    oe, og = make_optimizer(pe, capturable=True), make_optimizer(pg, capturable=True)
    se = ppo_epochs(pe, oe, states, acts, logp, vals, ret, adv, epochs=2, batch_size=bs,
                    generator=torch.Generator().manual_seed(7))
    up = GraphPPOUpdater(pg, og, states, acts, logp, vals, ret, adv, bs)
    sg = up.run(epochs=2, generator=torch.Generator().manual_seed(7))
    assert se[3] == sg[3] == 2 * (n // bs)
    np.testing.assert_allclose(sg[:3], se[:3], rtol=1e-5, atol=1e-6)
    for (k, a), b in zip(pe.state_dict().items(), pg.state_dict().values()):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.parametrize("E,N,M,period", [(4096, 16, 32, 3), (1000, 8, 16, 2), (96, 64, 64, 0), (33, 4, 4, 5)])
def test_fused_rollout_step_matches_two_launches(E, N, M, period):
    """uavhip_rollout_step (window-row forward + sampling + env step in one launch) against the
    separate policy and env launches it replaces (each checked against the reference above), and
    uavhip_rollout_steps (all T steps of an iteration in one launch) against both, on triplet envs
    from the same seed: every trajectory output, the row cache and the whole env state bitwise
    over two iterations with auto-reset and full resets flipping to refreshed scenes."""
    from uavhip.policy import TransformerActorCritic
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv
    torch.manual_seed(0)
    pol = TransformerActorCritic().cuda()
    T = 20
    res = []
    for fused, persistent in ((False, False), (True, False), (True, True)):
        env = VecUAVEnv(E, N, M, 1, 1, seed=6, full_reset_period=period)
        eng = RolloutEngine(env, pol, T, seed=5, fused_step=fused, persistent=persistent)
        assert eng.fused_step == fused and eng.persistent == persistent
        eng.start()
        out = []
        for _ in range(2):
            tr = eng.collect()
            out += [x.clone() for x in (tr.obs, tr.actions, tr.logp, tr.values, tr.rewards, tr.dones, tr.info,
                                        tr.ret, tr.adv, tr.last_values)]
        out += [eng.rowproj.clone(), env.istate.clone(), env.dstate.clone(), env.window.clone(), env.nh_final.clone(),
                env.nh_pure.clone(), env.t_cost.clone(), env.n_lock.clone(), env.assigned.clone()]
        assert int((env.errors() & 1).max()) == 0
        res.append(out)
    torch.cuda.synchronize()
    if N * M <= 512:
        assert res[1][5].any()  # episodes ended inside the rollout
    for i, (a, b, c) in enumerate(zip(*res)):
        assert torch.equal(a, b), i
        assert torch.equal(a, c), i


def test_fused_rollout_step_vs_oracle(traj_npz):
    """The rollout hot path against the CPU oracle directly: uavhip_rollout_step over the fixture
    scenes of one shape (several copies each, state-only auto-reset), every sampled action replayed
    through oracle.OracleEnv -- done flags bit-exact, rewards to 1e-12, next windows to the fp32 bar
    -- and logp / value against the torch forward of the same windows and actions."""
    import oracle
    from uavhip.policy import TransformerActorCritic, rowproj_buffer
    from uavhip.vec_env import VecUAVEnv
    groups = {}
    for c in cases(traj_npz):
        s = sub(traj_npz, c["key"])
        key = (c["N"], c["M"], len(s["nfz_pos"]), len(s["icp_pos"]), tuple(s["params"]))
        groups.setdefault(key, []).append(s)
    (N, M, Kn, Ki, prm), scenes = max(((k, g) for k, g in groups.items() if k[0] <= 64 and k[1] <= 64),
                                      key=lambda kv: kv[0][0] * kv[0][1] * len(kv[1]))
    scenes = (scenes * 8)[:48]
    E = len(scenes)
    torch.manual_seed(2)
    net = TransformerActorCritic().cuda()
    v = VecUAVEnv(E, N, M, Kn, Ki, full_reset_period=0)
    v.set_params(np.array(prm))
    v.load_scenes(scenes)
    obs = v.reset(episode=1).clone()
    refs = [oracle.OracleEnv(sc, np.array(prm)) for sc in scenes]
    for r in refs:
        r.reset()
    rp = rowproj_buffer(E)
    net.packed_weights()
    n_done = 0
    for t in range(40):
        act = torch.empty(E, dtype=torch.int8, device="cuda")
        lp, val = torch.empty(E, device="cuda"), torch.empty(E, device="cuda")
        nxt = torch.empty_like(obs)
        rew = torch.empty(E, dtype=torch.float64, device="cuda")
        dn = torch.empty(E, dtype=torch.uint8, device="cuda")
        net.rollout_step(v, obs, rp, t, t == 0, act, lp, val, nxt, rew, dn, seed=9, offset=t * E)
        with torch.no_grad():
            lp_t, v_t, _ = net.evaluate(obs, act.long())
        torch.testing.assert_close(lp, lp_t, rtol=1e-5, atol=2e-6)
        torch.testing.assert_close(val, v_t[:, 0], rtol=1e-5, atol=1e-5)
        a_h, r_h, d_h, o_h = act.cpu().numpy(), rew.cpu().numpy(), dn.cpu().numpy(), nxt.cpu().numpy()
        for e in range(E):
            o_c, r_c, d_c, _ = refs[e].step(int(a_h[e]))
            assert bool(d_h[e]) == d_c, (t, e)
            assert abs(r_h[e] - r_c) <= 1e-12 * max(1.0, abs(r_c)), (t, e, r_h[e], r_c)
            if d_c:
                n_done += 1
                o_c = refs[e].reset()
            np.testing.assert_allclose(o_h[e], o_c, rtol=2e-6, atol=1e-6)
        obs = nxt
    assert n_done > 0


@pytest.mark.parametrize("scale", [1.0, 40.0, 400.0, 4000.0])
def test_fused_forward_large_activations(policy_npz, scale):
    """Dynamic range of the split-product forward: the critic's layer-0 FFN1
    weight and bias scaled so the FFN hidden activations -- the FFN2 GEMM's split operand -- reach
    1.4e2 .. 1.4e4 (measured on MI355X, r04b: 3.6 at scale 1); the fused forward still matches the torch fp32 module to the
    usual bars (the split planes are 2^-22 relative anywhere in [2^-14, 65504])."""
    net = _load_policy(policy_npz, "b")
    lin = net.critic_net.transformer.layers[0].linear1
    with torch.no_grad():
        lin.weight.mul_(scale)
        lin.bias.mul_(scale)
    g = torch.Generator().manual_seed(7)
    x = (torch.randn(256, 5, 14, generator=g) * 0.7).cuda()
    a = torch.randint(0, 2, (256,), generator=g).cuda()
    hid = {}
    h = lin.register_forward_hook(lambda m, i, o: hid.__setitem__("max", float(o.relu().abs().max())))
    with torch.no_grad():
        logp_t, v_t, _ = net.evaluate(x, a)
    h.remove()
    print(f"scale {scale}: FFN hidden max {hid['max']:.3e}")
    _, logp, value, _, _ = net.fused_forward(x, actions=a)
    assert_close_report(f"scale {scale} logp", logp.cpu().numpy(), logp_t.cpu().numpy(), rtol=1e-5, atol=2e-6)
    assert_close_report(f"scale {scale} value", value.cpu().numpy(), v_t[:, 0].cpu().numpy(), rtol=1e-5, atol=1e-5)


def _range_case(net, case):
    """Drive one operand class of the split products out of fp16's normal range (policy_layout.hpp's
    range table must keep it exact): returns the input scale for the windows."""
    c0 = net.critic_net.transformer.layers[0]
    with torch.no_grad():
        if case.startswith("ffn1 x"):  # the critic's layer-0 FFN hidden units (FFN2's operand) to ~1.4e5
            k = float(case[len("ffn1 x"):])
            c0.linear1.weight.mul_(k)
            c0.linear1.bias.mul_(k)
        elif case == "ln1 x3e5":  # LN1's output (FFN1's operand) ~3e5 and the FFN hidden units ~1e6
            c0.norm1.weight.mul_(3e5)
            c0.norm1.bias.mul_(3e5)
        elif case == "ln1 x1e-6":  # LN1's output (FFN1's operand) ~1e-6; the FFN biases zero so it matters
            c0.norm1.weight.mul_(1e-6)
            c0.norm1.bias.mul_(1e-6)
            c0.linear1.bias.zero_()
            c0.linear2.bias.zero_()
        elif case == "inputs x1e5":  # every window row ~1e5: layer 0's input (e, e + pos) ~1e6
            return 1e5
        elif case == "inputs x1e-6":  # layer 0's input and attention output ~1e-6 (biases / pos zero)
            for tb in (net.actor_net, net.critic_net):
                tb.embedding[0].bias.zero_()
                tb.pos_embedding.zero_()
                tb.transformer.layers[0].self_attn.in_proj_bias.zero_()
                tb.transformer.layers[0].self_attn.out_proj.bias.zero_()
            return 1e-6
    return 1.0


RANGE_CASES = ["ffn1 x4e4", "ln1 x3e5", "ln1 x1e-6", "inputs x1e5", "inputs x1e-6"]


@pytest.mark.parametrize("case", RANGE_CASES)
def test_fused_forward_out_of_fp16_range_matches_torch(policy_npz, case):
    """every split-product operand is scaled by a power of two from a bound on its
    magnitude (policy_layout.hpp range table: per token for layer 0's input, per sample for layer 0's
    attention output, from the weights for the rest), so activations far outside fp16's normal range
    [2^-14, 65504] -- the critic's FFN hidden units at ~1.4e5 (FFN1 scaled; round 4 returned NaN here),
    LayerNorm outputs at ~3e5 with FFN hidden units at ~1e6, LayerNorm outputs at ~1e-6, window rows at
    1e5 and 1e-6 -- give the torch fp32
    module's logp / value / entropy within the usual bars (1e-5 relative), all finite. The full-window
    forward (uavhip_policy_forward) and the ring forward (uavhip_policy_forward_rows: fill + a
    shifted step) are both checked."""
    from uavhip.policy import rowproj_buffer
    net = _load_policy(policy_npz, "b")
    xs = _range_case(net, case)
    g = torch.Generator().manual_seed(8)
    x = (torch.randn(256, 5, 14, generator=g) * 0.7 * xs).cuda()
    x[:64, :2] = 0  # padded rows
    a = torch.randint(0, 2, (256,), generator=g).cuda()
    stats = {}
    lin = net.critic_net.transformer.layers[0].linear1
    h = lin.register_forward_hook(lambda m, i, o: stats.__setitem__("hid", float(o.relu().abs().max())))
    with torch.no_grad():
        logp_t, v_t, ent_t = net.evaluate(x, a)
    h.remove()
    print(f"{case}: critic FFN hidden max {stats['hid']:.3e}, |value| max {float(v_t.abs().max()):.3e}")
    assert torch.isfinite(v_t).all() and torch.isfinite(logp_t).all()
    _, logp, value, ent, _ = net.fused_forward(x, actions=a, entropy=torch.empty(256, device="cuda"))
    assert torch.isfinite(value).all() and torch.isfinite(logp).all(), "non-finite output"
    assert_close_report(f"{case} logp", logp.cpu().numpy(), logp_t.cpu().numpy(), rtol=1e-5, atol=2e-6)
    assert_close_report(f"{case} entropy", ent.cpu().numpy(), ent_t.cpu().numpy(), rtol=1e-5, atol=2e-6)
    assert_close_report(f"{case} value", value.cpu().numpy(), v_t[:, 0].cpu().numpy(), rtol=1e-5,
                        atol=1e-5 * max(1.0, float(v_t.abs().max())))
    # the ring forward: fill (rows 0-3 projected by k_policy_rows_fill) + the new row, then one step
    # along the window sequence (rows 0-3 from the ring)
    rp = rowproj_buffer(256)
    x1 = torch.cat([x[:, 1:], (torch.randn(256, 1, 14, generator=g) * 0.7 * xs).cuda()], 1)
    for step, xx in ((0, x), (1, x1)):
        with torch.no_grad():
            lp_t, vv_t, _ = net.evaluate(xx, a)
        _, lp, vv, _, _ = net.fused_forward(xx, actions=a, rowproj=rp, step=step, fill=step == 0)
        assert_close_report(f"{case} ring step {step} logp", lp.cpu().numpy(), lp_t.cpu().numpy(), rtol=1e-5,
                            atol=2e-6)
        assert_close_report(f"{case} ring step {step} value", vv.cpu().numpy(), vv_t[:, 0].cpu().numpy(), rtol=1e-5,
                            atol=1e-5 * max(1.0, float(vv_t.abs().max())))


ROLLOUT_RANGE_CASES = ["ffn1 x4e4", "rows x1e5", "rows x1e-6", "embed x1e5"]


@pytest.mark.parametrize("case", ROLLOUT_RANGE_CASES)
def test_rollout_steps_out_of_fp16_range_matches_torch(policy_npz, case):
    """the range scaling inside the headline kernel, k_rollout_steps (the
    RolloutEngine's one-launch-per-iteration path: ring fill, window-row forward with the range table
    and layer-0 constants staged in LDS once per launch, sampling, env step), T = 8 over 256 envs.
    Cases: the critic's layer-0 FFN1 x 4e4 (FFN hidden units ~1e5, FFN2's operand); window rows x 1e5
    and x 1e-6 (the env's window deque and the carried window scaled before the checked iteration, so
    steps 0-3 mix scaled rows -- read from the ring the fill projected -- with the env's new rows:
    per-token input exponents and the per-workgroup attention factor; for 1e-6 the embedding / position /
    in_proj / out_proj biases are zero so the small rows matter); the embeddings x 1e5 (every step's
    layer-0 input ~1e5 x). logp and value of every step against torch `evaluate` of the windows the
    kernel consumed (tr.obs[t]) with the actions it sampled: 1e-5 relative (transformer_net.py:124-144),
    or where torch fp32 is itself off the fp64 forward (mixed 1e5 / O(1) windows: attention logits
    ~1e10), within twice torch fp32's worst error of fp64 on the same case; all finite."""
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv
    net = _load_policy(policy_npz, "b")
    c0 = net.critic_net.transformer.layers[0]
    rows = 1.0
    with torch.no_grad():
        if case == "ffn1 x4e4":
            c0.linear1.weight.mul_(4e4)
            c0.linear1.bias.mul_(4e4)
        elif case == "embed x1e5":
            for tb in (net.actor_net, net.critic_net):
                tb.embedding[0].weight.mul_(1e5)
                tb.embedding[0].bias.mul_(1e5)
                tb.pos_embedding.mul_(1e5)
        elif case == "rows x1e5":
            rows = 1e5
        elif case == "rows x1e-6":
            rows = 1e-6
            for tb in (net.actor_net, net.critic_net):
                tb.embedding[0].bias.zero_()
                tb.pos_embedding.zero_()
                tb.transformer.layers[0].self_attn.in_proj_bias.zero_()
                tb.transformer.layers[0].self_attn.out_proj.bias.zero_()
    E, T = 256, 8
    env = VecUAVEnv(E, 16, 32, 1, 1, full_reset_period=200, seed=31)
    eng = RolloutEngine(env, net, T, seed=32)
    assert eng.persistent, "the test is of k_rollout_steps"
    eng.start()
    eng.collect()  # one iteration first: the windows are full (no padding) when they are scaled
    if rows != 1.0:
        with torch.no_grad():
            env.window.mul_(rows)
            eng.traj.obs[T].mul_(rows)
    tr = eng.collect()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.logp).all() and torch.isfinite(tr.values).all(), "non-finite output"
    x = tr.obs[:T].reshape(T * E, 5, 14)
    a = tr.actions.reshape(-1).long()
    if rows != 1.0:  # the scaled rows really were consumed: step 0's window holds them
        big = float(tr.obs[0].abs().amax())
        print(f"{case}: step-0 window max |x| {big:.3e}, step-{T - 1} window max |x| {float(tr.obs[T - 1].abs().amax()):.3e}")
        assert (big > 1e3) if rows > 1 else (big < 1e-3)
    import copy
    with torch.no_grad():
        lp_t, v_t, _ = net.evaluate(x, a)
        lp_64, v_64, _ = copy.deepcopy(net).double().cpu().evaluate(x.double().cpu(), a.cpu())
    assert torch.isfinite(lp_t).all() and torch.isfinite(v_t).all()
    got = {"logp": tr.logp.reshape(-1).double().cpu(), "value": tr.values.reshape(-1).double().cpu()}
    f32 = {"logp": lp_t.double().cpu(), "value": v_t[:, 0].double().cpu()}
    f64 = {"logp": lp_64, "value": v_64[:, 0]}
    for k, atol in (("logp", 2e-6), ("value", 1e-5 * max(1.0, float(v_t.abs().max())))):
        # 1e-5 relative against torch fp32 -- or, where that fails, no further from the fp64 forward than
        # twice torch fp32's worst error on the same case: windows mixing 1e5-scale rows with O(1) rows
        # give attention logits ~1e10, where fp32 rounding moves the softmax itself (torch fp32 included)
        bar = 1e-5 * f32[k].abs() + atol
        e_hip, e_t32 = (got[k] - f64[k]).abs(), (f32[k] - f64[k]).abs()
        near = (got[k] - f32[k]).abs() <= bar
        ok = near | (e_hip <= 2 * float(e_t32.max()) + atol)
        print(f"{case} rollout {k}: max |HIP - torch fp32| / bar {float(((got[k] - f32[k]).abs() / bar).max()):.3e} "
              f"({int((~near).sum())} of {near.numel()} beyond); vs fp64: HIP max {float(e_hip.max()):.3e} "
              f"p99 {float(e_hip.quantile(0.99)):.3e}, torch fp32 max {float(e_t32.max()):.3e} "
              f"p99 {float(e_t32.quantile(0.99)):.3e}")
        assert bool(ok.all()), f"{case} {k}: {int((~ok).sum())} elements beyond both bars"
