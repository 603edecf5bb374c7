"""GPU: the Python surface the reference's driver calls (UAVEnv.reset / step,
PPOAgent.select_action / store_transition / update, the buffer-length gate, policy_old.get_action,
policy.state_dict) driven by tests/dropin_app/boundary_driver.py through the drop-in launcher
`python -m uavhip.run_reference`, from a directory that also holds decoy copies of the reference's
packages: every import resolves to the drop-ins, episodes step the HIP env and the fused policy,
PPOAgent.update runs the HIP training step (one captured hipGraph per epoch), and the state_dict
checkpoint has the reference's 50 keys."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import PKG, ROOT, dropin_env, has_gpu, make_decoy_app

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]


def test_boundary_calls_through_launcher(tmp_path):
    script = open(os.path.join(ROOT, "tests", "dropin_app", "boundary_driver.py")).read()
    app = make_decoy_app(tmp_path, script)
    out = subprocess.run([sys.executable, "-u", "-m", "uavhip.run_reference", "main_train.py", "--episodes", "20"],
                         cwd=app, env=dropin_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    for mod, path in rep["modules"].items():
        assert os.path.abspath(path).startswith(PKG + os.sep), (mod, path)
    assert rep["episodes"] == 20 and rep["updates"] >= 1 and rep["steps"] >= 20 * 30  # >= N steps per episode
    assert rep["terminal_shapes"] == [[14]]  # the reference's terminal obs is zeros(14) (uav_env.py:188-189)
    assert all(np.isfinite(list(rep["last_stats"].values())))
    assert all(np.isfinite(rep["rewards"])) and min(rep["rewards"]) >= 0.0
    sd = torch.load(app / rep["checkpoint"], weights_only=True)
    assert len(sd) == 50 and sum(v.numel() for v in sd.values()) == 419267
