"""Drop-in for the reference's agents/ppo.py."""
from uavhip.ppo import PPOAgent  # noqa: F401
