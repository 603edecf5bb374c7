"""GPU: distributional parity of the on-device scene generator (uavhip_scene_generate, Philox4x32)
with the reference's _generate_scene (envs/uav_env.py:65-173).

131,072 device scenes at 16 UAVs x 32 targets (BASELINE configs[2]) against
  * the distributions the reference draws from (Kolmogorov-Smirnov for every continuous draw,
    chi-square for the discrete ones), and
  * two-sample, the bit-exact host generator uavhip/scene.py, which replays the reference's own
    numpy MT19937 / `random` call order (pinned to 48 reference scenes in test_host.py): 4,000 scenes.
Covered: the n2 ~ U{1..n_remain} draw (:125), the value multiset and its placement under the target
shuffle (:127-129,173), the target list-order permutation (:173), type-2 UAV placement under
random.shuffle (:81-84), UAV position / speed / heading (:86-110), target position / velocity
(:131-142), NFZ (:146-153) and interceptor (:156-170) draws, and independence across envs.
Significance 1e-4 per statistic (seeded streams: a run is deterministic)."""
import random

import numpy as np
import pytest
import torch
from scipy import stats

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]

E, N, M = 131072, 16, 32
H = 4000
ALPHA = 1e-4


@pytest.fixture(scope="module")
def dev():
    from uavhip.vec_env import VecUAVEnv
    v = VecUAVEnv(E, N, M, 1, 1, seed=2024, full_reset_period=0)
    v.generate_scenes()
    torch.cuda.synchronize()
    out = {k: getattr(v, k).cpu().numpy() for k in ("uav_pos", "uav_vel", "uav_load", "uav_cost", "uav_type",
                                                     "tgt_pos", "tgt_vel", "tgt_value", "tgt_id", "nfz_pos",
                                                     "icp_pos", "icp_vel")}
    del v
    torch.cuda.empty_cache()
    return out


@pytest.fixture(scope="module")
def host():
    from uavhip.config import Config
    from uavhip.scene import generate_scene
    c = Config()
    c.NUM_UAVS, c.NUM_TARGETS = N, M
    np.random.seed(7)
    random.seed(7)
    sc = [generate_scene(c) for _ in range(H)]
    return {k: np.stack([s[k] for s in sc]) for k in sc[0] if k != "total_swarm_cost"}


def ks(name, x, cdf_or_sample):
    p = stats.kstest(np.ravel(x), cdf_or_sample).pvalue
    print(f"{name}: KS p = {p:.3g}")
    assert p > ALPHA, name


def chi2(name, counts, expected):
    counts, expected = np.asarray(counts, float), np.asarray(expected, float)
    p = stats.chisquare(counts, expected * counts.sum() / expected.sum()).pvalue
    print(f"{name}: chi2 p = {p:.3g}")
    assert p > ALPHA, name


def two_sample(name, a, b):
    p = stats.ks_2samp(np.ravel(a), np.ravel(b)).pvalue
    print(f"{name}: two-sample KS vs host p = {p:.3g}")
    assert p > ALPHA, name


def uniform(lo, hi):
    return stats.uniform(lo, hi - lo).cdf


def test_target_values_and_n2(dev, host):
    n1, n_remain = M // 2, M - M // 2 - 1
    for s in (dev, host):
        tv = s["tgt_value"]
        assert ((tv == 4).sum(1) == n1).all() and ((tv == 16).sum(1) == 1).all()
        assert ((tv == 6).sum(1) + (tv == 8).sum(1) == n_remain).all()
    n2_dev = (dev["tgt_value"] == 6).sum(1)
    assert n2_dev.min() >= 1 and n2_dev.max() <= n_remain
    chi2("n2 ~ U{1..n_remain}", np.bincount(n2_dev, minlength=n_remain + 1)[1:], np.ones(n_remain))
    n2_host = (host["tgt_value"] == 6).sum(1)
    tab = np.stack([np.bincount(n2_dev, minlength=n_remain + 1)[1:], np.bincount(n2_host, minlength=n_remain + 1)[1:]])
    p = stats.chi2_contingency(tab).pvalue
    print(f"n2 device vs host: chi2 p = {p:.3g}")
    assert p > ALPHA


def test_target_shuffle(dev, host):
    tid, tv = dev["tgt_id"], dev["tgt_value"]
    assert (np.sort(tid, 1) == np.arange(M)).all()  # a permutation of the pre-shuffle ids
    # list position of id 0, of the 16-value target, and the id at list position 0: uniform
    chi2("position of id 0", np.bincount(np.argmax(tid == 0, 1), minlength=M), np.ones(M))
    chi2("position of the 16-value target", np.bincount(np.argmax(tv == 16, 1), minlength=M), np.ones(M))
    chi2("id at position 0", np.bincount(tid[:, 0], minlength=M), np.ones(M))
    # pairwise order of two positions: fair
    chi2("id[0] < id[1]", np.bincount((tid[:, 0] < tid[:, 1]).astype(int), minlength=2), np.ones(2))
    # value and id independent (values shuffled before the targets, :127 and :173)
    cls = np.searchsorted([4, 6, 8, 16], tv[:, :4].ravel())
    p = stats.chi2_contingency(np.histogram2d(cls, tid[:, :4].ravel(), bins=[4, M])[0]).pvalue
    print(f"value class x id: chi2 p = {p:.3g}")
    assert p > ALPHA
    # the host generator's placement of the 16-value target agrees
    tab = np.stack([np.bincount(np.argmax(tv == 16, 1), minlength=M),
                    np.bincount(np.argmax(host["tgt_value"] == 16, 1), minlength=M)])
    assert stats.chi2_contingency(tab).pvalue > ALPHA


def test_uav_types_and_kinematics(dev, host):
    ut = dev["uav_type"]
    assert ((ut == 2).sum(1) == N // 4).all()
    chi2("type-2 UAV index", (ut == 2).sum(0), np.ones(N))
    both = ((ut[:, 0] == 2) & (ut[:, 1] == 2)).mean()
    expect = (N // 4) / N * (N // 4 - 1) / (N - 1)  # random.shuffle: a uniform permutation
    assert abs(both - expect) < 5 * np.sqrt(expect * (1 - expect) / E)
    for s, tag in ((dev, "device"), (host, "host")):
        np.testing.assert_array_equal(s["uav_cost"], np.where(s["uav_type"] == 1, 1.0, 1.25))
        np.testing.assert_array_equal(s["uav_load"], np.where(s["uav_type"] == 1, 0.95, 1.0))
    up, uv = dev["uav_pos"], dev["uav_vel"]
    sp = np.linalg.norm(uv, axis=-1)
    hd = np.degrees(np.arctan2(uv[..., 1], uv[..., 0]))
    ks("UAV x", up[..., 0], uniform(60, 90))
    ks("UAV y", up[..., 1], uniform(0, 160))
    ks("type-1 speed", sp[ut == 1], uniform(0.35, 0.50))
    ks("type-2 speed", sp[ut == 2], uniform(0.75, 0.90))
    ks("heading (deg)", hd, uniform(-15, 15))
    hs = np.linalg.norm(host["uav_vel"], axis=-1)
    two_sample("UAV x", up[..., 0], host["uav_pos"][..., 0])
    two_sample("type-1 speed", sp[ut == 1], hs[host["uav_type"] == 1])
    two_sample("heading", hd, np.degrees(np.arctan2(host["uav_vel"][..., 1], host["uav_vel"][..., 0])))


def test_targets_obstacles_interceptors(dev, host):
    tp, tvel = dev["tgt_pos"], dev["tgt_vel"]
    ks("target x", tp[..., 0], uniform(160, 180))
    ks("target y", tp[..., 1], uniform(0, 160))
    ks("target vx", tvel[..., 0], uniform(-0.015, 0.015))
    ks("target vy", tvel[..., 1], uniform(-0.015, 0.015))
    two_sample("target vx", tvel[..., 0], host["tgt_vel"][..., 0])
    two_sample("target y", tp[..., 1], host["tgt_pos"][..., 1])
    ks("NFZ x", dev["nfz_pos"][:, 0, 0], uniform(120, 140))
    ks("NFZ y", dev["nfz_pos"][:, 0, 1], uniform(0, 160))
    ip, iv = dev["icp_pos"][:, 0], dev["icp_vel"][:, 0]
    ks("interceptor x", ip[:, 0], uniform(140, 160))
    ks("interceptor y", ip[:, 1], uniform(0, 160))
    ks("interceptor speed", np.linalg.norm(iv, axis=-1), uniform(0.30, 0.32))
    ks("interceptor heading", np.mod(np.arctan2(iv[:, 1], iv[:, 0]), 2 * np.pi), uniform(0, 2 * np.pi))
    two_sample("interceptor speed", np.linalg.norm(iv, axis=-1), np.linalg.norm(host["icp_vel"][:, 0], axis=-1))
    two_sample("NFZ x", dev["nfz_pos"][:, 0, 0], host["nfz_pos"][:, 0, 0])


def test_envs_independent(dev):
    """Neighbouring envs (consecutive Philox counters) are uncorrelated, and no two scenes repeat."""
    x = dev["uav_pos"][:, 0, 0]
    r = np.corrcoef(x[:-1], x[1:])[0, 1]
    assert abs(r) < 5 / np.sqrt(E), r
    y = dev["tgt_pos"][:, 0, 1]
    assert abs(np.corrcoef(y[::2], y[1::2])[0, 1]) < 5 / np.sqrt(E / 2)
    assert len(np.unique(dev["uav_pos"][:, :2].reshape(E, -1), axis=0)) == E
