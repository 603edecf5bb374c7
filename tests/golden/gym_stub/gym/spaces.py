"""`gym.spaces` stand-in: records constructor arguments, nothing else."""


class Discrete:
    def __init__(self, n, *args, **kwargs):
        self.n = n


class Box:
    def __init__(self, low=None, high=None, shape=None, dtype=None, *args, **kwargs):
        self.low, self.high, self.shape, self.dtype = low, high, shape, dtype
