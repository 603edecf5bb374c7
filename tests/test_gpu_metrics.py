"""GPU: device episode statistics (uavhip_episode_stats, main_train.py:118-137 accumulation) vs
the plain-Python restatement in oracle/metrics.py, over two rollout chunks of the real engine
(episodes carried across the chunk boundary). Sums are in step order in fp64 on both sides:
records must match exactly."""
import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]


def test_episode_stats_match_restatement():
    from oracle import metrics as om
    from uavhip.metrics import EpisodeStats, csv_rows
    from uavhip.policy import TransformerActorCritic
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv
    torch.manual_seed(0)
    env = VecUAVEnv(96, 6, 8, 1, 1, seed=3, full_reset_period=4)
    pol = TransformerActorCritic().cuda()
    eng = RolloutEngine(env, pol, 40, want_info=True, seed=5)
    eng.start()
    st = EpisodeStats(96)
    acc = None
    recs = []
    for _ in range(2):
        tr = eng.collect(eager=True)
        st.update(tr)
        r, acc = om.episode_records(tr.rewards.cpu().numpy(), tr.dones.cpu().numpy(), tr.actions.cpu().numpy(),
                                    tr.info.cpu().numpy(), tr.values.cpu().numpy(), acc)
        recs.append(r)
    ref = np.concatenate(recs)
    ref = ref[np.lexsort((ref[:, 1], ref[:, 0]))]
    got = st.drain()
    assert len(got) == len(ref) > 50
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(st.acc.cpu().numpy(), acc)
    rows = csv_rows(got)
    assert len(rows) == len(got) and len(rows[0]) == 12


def test_episode_stats_match_main_train():
    """uavhip_episode_stats against the reference's own main_train.train() (tests/golden/main_train.npz,
    30 episodes): the per-step info stream as one env's rollout chunks (split at an arbitrary step, so
    the open episode carries across the chunk boundary) gives exactly the accumulators train() held."""
    from conftest import load_golden, main_train_chunk, main_train_records
    from uavhip.metrics import EpisodeStats
    mt = load_golden("main_train.npz")
    rew, done, act, info, val = main_train_chunk(mt)
    st = EpisodeStats(1)
    cut = len(rew) // 2 + 7
    for sl in (slice(0, cut), slice(cut, None)):
        tr = type("Chunk", (), {})()
        tr.rewards, tr.dones, tr.actions = (torch.from_numpy(np.ascontiguousarray(x[sl])).cuda() for x in (rew, done, act))
        tr.info = torch.from_numpy(np.ascontiguousarray(info[sl])).cuda()
        tr.values = torch.from_numpy(np.ascontiguousarray(val[sl])).cuda()
        st.update(tr)
    got = st.drain()
    np.testing.assert_array_equal(got, main_train_records(mt))
    assert not st.acc.any()
