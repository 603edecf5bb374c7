"""ORACLE (test infrastructure): numpy fp32 restatement of agents/ppo.py:70-94.

Op-by-op float32, in the reference's evaluation order:
  values = cat(values).squeeze()                              ppo.py:72
  next_values = cat(values[1:], [0.0])                        ppo.py:77
  for t reversed:                                             ppo.py:81-89
      v_next = next_values[t] if not done else 0.0
      delta  = r_t + GAMMA * v_next - v_t       (r_t: python f64 -> cast to f32 by the tensor op)
      gae    = delta + GAMMA*LAMBDA * gae * (1 - done)   (GAMMA*LAMBDA is an f64 product, cast once)
      returns[t] = gae + v_t
  advantages = returns - values                               ppo.py:91
  advantages = (adv - adv.mean()) / (adv.std() + 1e-7)        ppo.py:94 (unbiased std)
The mean/std here are formed in float64 and rounded to float32 (torch CPU uses its own
reduction order), so normalised advantages agree to ~1e-7 relative, returns bit-exactly.
"""
import numpy as np

f32 = np.float32


def gae_1d(rewards, dones, values, gamma=0.998, lam=0.95, last_value=None):
    """One concatenated buffer (the reference's layout). Returns (returns, advantages) f32."""
    r = np.asarray(rewards, np.float64)
    d = np.asarray(dones).astype(bool)
    v = np.asarray(values, np.float32)
    T = len(v)
    nv = np.empty(T, np.float32)
    nv[:-1] = v[1:]
    nv[-1] = f32(0.0) if last_value is None else f32(last_value)
    g = f32(gamma)
    gl = f32(gamma * lam)
    gae = f32(0.0)
    ret = np.empty(T, np.float32)
    for t in range(T - 1, -1, -1):
        rt = f32(r[t])
        if d[t]:
            delta = f32(rt - v[t])
            gae = delta
        else:
            delta = f32(f32(rt + f32(g * nv[t])) - v[t])
            gae = f32(delta + f32(gl * gae))
        ret[t] = f32(gae + v[t])
    adv = (ret - v).astype(np.float32)
    return ret, adv


def gae_2d(rewards, dones, values, gamma=0.998, lam=0.95, last_values=None):
    """Vectorised layout [T, E] (time-major): each env column is an independent buffer."""
    rewards = np.asarray(rewards); dones = np.asarray(dones); values = np.asarray(values, np.float32)
    T, E = values.shape
    ret = np.empty((T, E), np.float32); adv = np.empty((T, E), np.float32)
    for e in range(E):
        lv = None if last_values is None else last_values[e]
        ret[:, e], adv[:, e] = gae_1d(rewards[:, e], dones[:, e], values[:, e], gamma, lam, lv)
    return ret, adv


def normalize(adv):
    a = np.asarray(adv, np.float32)
    a64 = a.astype(np.float64)
    mean = f32(a64.mean())
    std = f32(a64.std(ddof=1)) if a.size > 1 else f32(np.nan)
    return ((a - mean) / f32(std + f32(1e-7))).astype(np.float32), float(mean), float(std)
