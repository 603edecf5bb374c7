"""Training-curve statistics of main_train.py (:122-136 per-step accumulation, :161-195 the CSV
columns) for the batched rollout: `EpisodeStats.update(traj)` runs uavhip_episode_stats over a
rollout chunk on the device (episodes carry across chunks), `drain()` returns the finished
episodes' records and `csv_rows` turns them into main_train's CSV columns.
"""
import numpy as np
import torch

from . import _lib
from ._lib import LIB, check, ptr, stream_handle

CSV_HEADER = ["Episode", "Avg_Reward", "Avg_Q0", "Avg_J_Value", "Max_Coverage", "Action1_Ratio",
              "Valid_Assign_Rate", "Avg_P_Dmg", "Avg_P_Final", "Loss_Critic", "Loss_Actor", "Entropy"]


class EpisodeStats:
    def __init__(self, num_envs, device="cuda", max_records=1 << 16):
        self.E, self.max_records = int(num_envs), int(max_records)
        f64 = dict(dtype=torch.float64, device=device)
        self.acc = torch.zeros(self.E, _lib.EP_COUNT, **f64)
        self.records = torch.zeros(self.max_records, _lib.EP_COUNT, **f64)
        self.count = torch.zeros(1, dtype=torch.int32, device=device)
        self.dropped = 0

    def update(self, traj):
        """Accumulate one rollout chunk (uavhip.rollout.Trajectory with info)."""
        if traj.info is None:
            raise ValueError("episode statistics need the rollout's info buffer (want_info=True)")
        T, E = traj.actions.shape
        check(LIB.uavhip_episode_stats(ptr(traj.rewards), ptr(traj.dones), ptr(traj.actions), ptr(traj.info),
                                       ptr(traj.values), T, E, ptr(self.acc), ptr(self.records), self.max_records,
                                       ptr(self.count), stream_handle()), "uavhip_episode_stats")

    def drain(self):
        """Finished episodes since the last drain, [n][EP_COUNT] float64 sorted by (env, episode)."""
        n = int(self.count.item())
        kept = min(n, self.max_records)
        self.dropped += n - kept
        rec = self.records[:kept].cpu().numpy().copy()
        self.count.zero_()
        return rec[np.lexsort((rec[:, _lib.EP["EPISODE"]], rec[:, _lib.EP["ENV"]]))]


def derived(rec):
    """main_train.py:165-173 per-episode quantities from records -> dict of arrays."""
    E = _lib.EP
    steps = np.maximum(1.0, rec[:, E["STEPS"]])
    act1 = rec[:, E["ACTION1"]]
    asg = np.maximum(1.0, rec[:, E["ASSIGN_STEPS"]])
    return {"reward": rec[:, E["REWARD"]], "q0": rec[:, E["Q0"]], "avg_J": rec[:, E["J_SUM"]] / steps,
            "max_cov": rec[:, E["MAX_COV"]], "action1_ratio": act1 / steps,
            "valid_rate": rec[:, E["VALID"]] / np.maximum(1.0, act1),
            "avg_p_dmg": rec[:, E["PDMG_SUM"]] / asg, "avg_p_final": rec[:, E["PFINAL_SUM"]] / asg}


def csv_rows(rec, first_episode=1, window=50, losses=(0.0, 0.0, 0.0)):
    """One CSV row per record in the given order, columns as main_train.py:56-61 (Avg_Reward and
    Avg_Q0 are moving averages over the last `window` episodes, :146-157). losses: (critic, actor,
    entropy) of the update behind every row (main_train.py:176-178; zeros when none ran), or one
    such triple per record."""
    d = derived(rec)
    per_row = np.ndim(losses) == 2
    rows = []
    for i in range(len(rec)):
        lo = max(0, i + 1 - window)
        lc, la, le = losses[i] if per_row else losses
        rows.append([first_episode + i, f"{np.mean(d['reward'][lo:i + 1]):.4f}", f"{np.mean(d['q0'][lo:i + 1]):.4f}",
                     f"{d['avg_J'][i]:.4f}", int(d["max_cov"][i]), f"{d['action1_ratio'][i]:.4f}",
                     f"{d['valid_rate'][i]:.4f}", f"{d['avg_p_dmg'][i]:.4f}", f"{d['avg_p_final'][i]:.4f}",
                     f"{lc:.6f}", f"{la:.6f}", f"{le:.6f}"])
    return rows
