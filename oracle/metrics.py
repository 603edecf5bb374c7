"""CPU restatement (test infrastructure, not product) of main_train.py's per-episode statistic
accumulation (main_train.py:122-136): plain Python loops over a [T][E] rollout chunk, one env at a
time in step order, the sums in Python floats (fp64) as the reference's. Used only by tests."""
import numpy as np

# record layout = include/uavhip.h enum uavhip_ep
COUNT = 12


def episode_records(rewards, dones, actions, info, values, acc=None):
    """-> (records [n][12] in (env, episode) order, acc [E][12] of unfinished episodes).
    info columns: J=0, NUM_ASSIGNED=1, IS_VALID=2 (1/0, -1 = None), AVG_P_DMG=3, AVG_P_FINAL=4,
    EPISODE=7 (include/uavhip.h enum uavhip_info)."""
    T, E = actions.shape
    acc = np.zeros((E, COUNT)) if acc is None else acc.copy()
    out = []
    for e in range(E):
        a = [float(x) for x in acc[e]]
        for t in range(T):
            if a[2] == 0.0:
                a[4] = float(values[t, e])                 # current_q0 (main_train.py:87-93)
            inf = info[t, e]
            a[2] += 1.0                                     # ep_steps += 1 (:125)
            a[3] = a[3] + float(rewards[t, e])              # current_ep_reward += reward (:122)
            a[5] = a[5] + float(inf[0])                     # ep_total_J += J_val (:127)
            a[6] = max(a[6], float(inf[1]))                 # ep_max_cov (:128)
            if int(actions[t, e]) == 1:                     # :130-133
                a[7] += 1.0
                if inf[2] == 1.0:
                    a[8] += 1.0
            if inf[1] > 0:                                  # :134-137
                a[9] = a[9] + float(inf[3])
                a[10] = a[10] + float(inf[4])
                a[11] += 1.0
            if dones[t, e]:
                a[0], a[1] = float(e), float(inf[7])
                out.append(list(a))
                a = [0.0] * COUNT
        acc[e] = a
    rec = np.array(out, dtype=np.float64).reshape(-1, COUNT)
    return rec, acc
