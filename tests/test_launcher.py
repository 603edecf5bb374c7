"""The drop-in launcher (uavhip.run_reference). A script whose own
directory holds decoy copies of the reference's packages (configs / envs / agents / networks, raising
on import) must import the drop-ins when run through the launcher -- with its argv, __name__ and
working directory as if run directly. Control: run directly with only PYTHONPATH set, the same
script imports the decoys (Python puts the script's directory ahead of PYTHONPATH), which is why
the launcher exists. CPU only (the drop-ins import without a GPU; nothing is computed)."""
import json
import os
import subprocess
import sys
import textwrap

from conftest import PKG, dropin_env, make_decoy_app

SCRIPT = textwrap.dedent('''
    import json, os, sys
    from configs.config import cfg
    import envs.entities
    from envs.uav_env import UAVEnv
    from agents.ppo import PPOAgent
    from networks.transformer_net import TransformerActorCritic
    mods = {m: sys.modules[m].__file__ for m in ("configs.config", "envs.entities", "envs.uav_env", "agents.ppo",
                                                 "networks.transformer_net")}
    print(json.dumps({"mods": mods, "argv": sys.argv[1:], "name": __name__, "cwd": os.getcwd(),
                      "batch": cfg.BATCH_SIZE, "classes": [UAVEnv.__name__, PPOAgent.__name__,
                                                           TransformerActorCritic.__name__]}))
''')


def test_launcher_imports_dropins_over_the_script_directory(tmp_path):
    app = make_decoy_app(tmp_path, SCRIPT)
    out = subprocess.run([sys.executable, "-m", "uavhip.run_reference", "main_train.py", "--episodes", "3"], cwd=app,
                         env=dropin_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    for mod, path in rep["mods"].items():
        assert os.path.abspath(path).startswith(PKG + os.sep), (mod, path)
    assert rep["argv"] == ["--episodes", "3"] and rep["name"] == "__main__"
    assert os.path.samefile(rep["cwd"], app) and rep["batch"] == 64
    assert rep["classes"] == ["UAVEnv", "PPOAgent", "TransformerActorCritic"]


def test_direct_run_imports_the_decoys(tmp_path):
    """Documents the failure the launcher fixes: PYTHONPATH alone loses to the script directory."""
    app = make_decoy_app(tmp_path, SCRIPT)
    out = subprocess.run([sys.executable, "main_train.py"], cwd=app, env=dropin_env(), capture_output=True, text=True,
                         timeout=300)
    assert out.returncode != 0 and "decoy reference module imported: configs.config" in out.stderr


def test_launcher_usage():
    out = subprocess.run([sys.executable, "-m", "uavhip.run_reference"], env=dropin_env(), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 2 and "usage" in out.stderr
