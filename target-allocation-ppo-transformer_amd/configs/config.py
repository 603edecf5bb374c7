"""Drop-in for the reference's configs/config.py: the shared `cfg` singleton."""
from uavhip.config import Config, cfg  # noqa: F401
