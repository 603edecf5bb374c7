"""Drop-in for the reference's envs/entities.py: the record types (entities.py:7-61). In this
build they are host-side views of the device SoA state (see envs/uav_env.py)."""
from dataclasses import dataclass, field
from typing import List

import numpy as np


@dataclass
class Entity:
    id: int
    pos: np.ndarray


@dataclass
class UAV(Entity):
    velocity: np.ndarray = field(default_factory=lambda: np.zeros(2))
    max_speed: float = 0.0
    load: float = 0.0
    uav_type: int = 1
    cost: float = 1.0
    assigned_target_id: int = -1
    available: bool = True

    def reset(self, pos, v, speed, load, cost=1.0):
        self.pos, self.velocity, self.max_speed, self.load, self.cost = pos, v, speed, load, cost
        self.assigned_target_id = -1
        self.available = True


@dataclass
class Target(Entity):
    value: float = 1.0
    defense_level: float = 0.0
    required_load: float = 0.0
    locked_by_uavs: List[int] = field(default_factory=list)
    velocity: np.ndarray = field(default_factory=lambda: np.zeros(2))

    def reset(self):
        self.locked_by_uavs = []


@dataclass
class NoFlyZone(Entity):
    radius: float = 1.0
    penalty_factor: float = 0.5


@dataclass
class Interceptor(Entity):
    radius: float = 2.0
    kill_prob: float = 0.3
    velocity: np.ndarray = field(default_factory=lambda: np.zeros(2))
