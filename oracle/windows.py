"""ORACLE (test infrastructure): numpy restatement of UAVEnv's observation window (the deque of
the last 5 state rows, envs/uav_env.py:42-63 reset -> zeros, :241-242 append) for rebuilding a
trajectory's policy inputs from the compact data-parallel exchange format (uavhip/dist.py):
the first window of each env, the row pushed at every step, and the done flags.

Step-by-step, exactly as the deque evolves: W(0) = first; W(t) = [0, 0, 0, 0, row(t)] if the
episode ended at step t - 1, else W(t - 1)[1:] + [row(t)].
"""
import numpy as np


def windows_from_rows(first, rows, dones):
    """first [E][5][14], rows [T][E][14] (row(t) = W(t)[4]), dones [T][E] -> windows [T][E][5][14]."""
    first = np.asarray(first, np.float32).reshape(-1, 5, 14)
    rows = np.asarray(rows, np.float32)
    dones = np.asarray(dones) != 0
    T, E = rows.shape[:2]
    out = np.zeros((T, E, 5, 14), np.float32)
    w = first.copy()
    for t in range(T):
        if t > 0:
            nxt = np.zeros_like(w)
            keep = ~dones[t - 1]
            nxt[keep, :4] = w[keep, 1:]
            nxt[:, 4] = rows[t]
            w = nxt
        out[t] = w
    return out
