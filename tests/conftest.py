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
