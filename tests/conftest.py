"""Shared test setup.

* registers the ``gpu`` marker (tests that need an MI355X; run with ``-m gpu``)
* puts the repo root (for ``oracle``) and the package directory
  ``target-allocation-ppo-transformer_amd/`` (for ``uavhip`` and the drop-in
  ``envs``/``agents``/``networks``/``configs`` modules) on sys.path
* loads the golden fixtures (tests/golden/*.npz, produced by the reference itself)
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "target-allocation-ppo-transformer_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def cases(npz):
    return json.loads(str(npz["manifest"]))["cases"]


def sub(npz, key):
    pre = key + "/"
    return {k[len(pre):]: npz[k] for k in npz.files if k.startswith(pre)}


@pytest.fixture(scope="session")
def traj_npz():
    return load_golden("traj.npz")


@pytest.fixture(scope="session")
def scenes_npz():
    return load_golden("scenes.npz")


@pytest.fixture(scope="session")
def mech_npz():
    return load_golden("mechanics.npz")


@pytest.fixture(scope="session")
def policy_npz():
    return load_golden("policy.npz")


@pytest.fixture(scope="session")
def gae_npz():
    return load_golden("gae.npz")


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


# ------------------------------------------------------------------ drop-in launcher apps
DECOY = 'raise ImportError("decoy reference module imported: {}")\n'
DECOY_MODULES = {"configs": ["config"], "envs": ["uav_env", "entities", "mechanics"], "agents": ["ppo"],
                 "networks": ["transformer_net"]}


def make_decoy_app(root, script_text, script_name="main_train.py"):
    """A directory laid out like the reference (configs/ envs/ agents/ networks/ next to the script)
    whose packages raise on import: a script run from it only works if the drop-ins win."""
    app = root / "ref"
    for pkg, mods in DECOY_MODULES.items():
        d = app / pkg
        d.mkdir(parents=True)
        (d / "__init__.py").write_text("")
        for m in mods:
            (d / f"{m}.py").write_text(DECOY.format(f"{pkg}.{m}"))
    (app / script_name).write_text(script_text)
    return app


def dropin_env():
    """Environment of a child process that has only PYTHONPATH pointing at the drop-in directory."""
    env = dict(os.environ)
    env["PYTHONPATH"] = PKG + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    return env


def assert_close_report(name, got, want, rtol, atol):
    """np.testing.assert_allclose that first prints the errors it measured (max |d|, max |d| / |want|
    over |want| > atol), so every bar can be read against the error it actually bounds."""
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    d = np.abs(got - want)
    big = np.abs(want) > atol
    rel = float((d[big] / np.abs(want[big])).max()) if big.any() else 0.0
    print(f"{name}: max |d| = {float(d.max()):.3e}, max rel = {rel:.3e} (bar rtol {rtol:g}, atol {atol:g})")
    np.testing.assert_allclose(got, want, rtol=rtol, atol=atol, err_msg=name)


def main_train_chunk(mt):
    """tests/golden/main_train.npz (the reference's main_train.train(), 30 episodes) as one env's
    [T, 1] rollout chunk in the layout of uavhip_episode_stats: rewards, dones, actions, info
    [T, 1, 8] (include/uavhip.h uavhip_info; EPISODE = the episode index), values (each episode's
    Q0, the reference's policy_old value of its first state, at every step: only the first is read)."""
    st, ep = mt["steps"], mt["episodes"]
    T = len(st)
    q0 = dict(zip(ep[:, 0].astype(int), ep[:, 2]))
    info = np.zeros((T, 1, 8))
    info[:, 0, 0], info[:, 0, 1], info[:, 0, 2], info[:, 0, 3], info[:, 0, 4] = st[:, 4], st[:, 5], st[:, 6], st[:, 7], st[:, 8]
    info[:, 0, 7] = st[:, 0]
    values = np.array([q0[int(e)] for e in st[:, 0]], np.float32).reshape(T, 1)
    return (st[:, 2].reshape(T, 1), st[:, 3].astype(np.uint8).reshape(T, 1), st[:, 1].astype(np.int8).reshape(T, 1),
            info, values)


def main_train_records(mt):
    """The reference's per-episode accumulators (main_train.py:98-136, read from train()'s frame) in
    the uavhip_ep record layout: ENV, EPISODE, STEPS, REWARD, Q0, J_SUM, MAX_COV, ACTION1, VALID,
    PDMG_SUM, PFINAL_SUM, ASSIGN_STEPS."""
    ep = mt["episodes"]  # episode, reward, q0, J, steps, max_cov, action1, valid, p_dmg, p_final, assign steps
    return np.stack([np.zeros(len(ep)), ep[:, 0], ep[:, 4], ep[:, 1], ep[:, 2], ep[:, 3], ep[:, 5], ep[:, 6], ep[:, 7],
                     ep[:, 8], ep[:, 9], ep[:, 10]], axis=1)
