"""Minimal stand-in for the `gym` package, used ONLY by tests/golden/make_golden.py.

The reference (`envs/uav_env.py:2,6,13,18-24`) subclasses `gym.Env` and builds
`spaces.Discrete` / `spaces.Box`; nothing on its hot path calls into gym. gym is
not installed in this image, so this stub supplies exactly those three names.
"""
from . import spaces  # noqa: F401


class Env:
    def __init__(self, *args, **kwargs):
        pass
