"""Run one of the reference's scripts (main_train.py, ...) on the MI355X drop-ins.

    PYTHONPATH=<repo>/target-allocation-ppo-transformer_amd \
        python -m uavhip.run_reference /path/to/reference/main_train.py [script args ...]

Why a launcher: `python main_train.py` puts the script's own directory at sys.path[0], ahead of
every PYTHONPATH entry, so `from envs.uav_env import UAVEnv` / `from agents.ppo import PPOAgent`
(main_train.py:8-10) would resolve to the reference's pure-Python modules sitting next to it. This
launcher puts the drop-in directory FIRST and the script's directory second (so the script's other
sibling imports still resolve), drops any already-imported module of the four shadowed packages that
does not come from the drop-ins, and runs the script as __main__ with runpy -- the same globals,
argv and working directory the script sees when it is run directly.
"""
import os
import runpy
import sys

DROPIN = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHADOWED = ("configs", "envs", "agents", "networks")


def _from_dropin(mod):
    f = getattr(mod, "__file__", None)
    return f is not None and os.path.abspath(f).startswith(DROPIN + os.sep)


def prepare(script):
    """sys.path / sys.modules such that `script`'s imports of configs / envs / agents / networks
    resolve to the drop-ins. Returns the script's absolute path."""
    script = os.path.abspath(script)
    sdir = os.path.dirname(script)
    rest = [p for p in sys.path if os.path.abspath(p or os.curdir) not in (DROPIN, sdir)]
    sys.path[:] = [DROPIN, sdir] + rest
    for name in list(sys.modules):
        if name.split(".")[0] in SHADOWED and not _from_dropin(sys.modules[name]):
            del sys.modules[name]
    return script


def run(script, argv=()):
    """Run `script` as __main__ on the drop-ins (argv = its command-line arguments)."""
    script = prepare(script)
    sys.argv = [script] + list(argv)
    return runpy.run_path(script, run_name="__main__")


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    if not argv or argv[0] in ("-h", "--help"):
        print("usage: python -m uavhip.run_reference SCRIPT [ARGS ...]", file=sys.stderr)
        return 2
    run(argv[0], argv[1:])
    return 0


if __name__ == "__main__":
    sys.exit(main())
