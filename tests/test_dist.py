"""Multi-process (world_size 2 and 3, gloo on CPU) checks of the data-parallel plumbing in
uavhip.dist: env sharding, the single trajectory all-gather (rank order, record layout) and the
global advantage moments all-reduce. The RCCL path runs the same functions with backend "nccl"."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "target-allocation-ppo-transformer_amd"))
    import torch.distributed as dist
    from uavhip import dist as udist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        T, E_total = 6, 10
        start, cnt = udist.shard(E_total, world, rank)
        g = torch.Generator().manual_seed(1000 + rank)
        obs = torch.randn(T, cnt, 5, 14, generator=g)
        actions = torch.randint(0, 2, (T, cnt), generator=g, dtype=torch.int8)
        f = [torch.randn(T, cnt, generator=g) for _ in range(4)]
        rewards = torch.rand(T, cnt, generator=g, dtype=torch.float64)
        dones = (torch.rand(T, cnt, generator=g) < 0.2).to(torch.uint8)
        payload = udist.pack_trajectory(obs, actions, f[0], f[1], f[2], f[3], rewards, dones)
        # equal-size payloads per rank (pad the smaller shard's rows for the collective)
        rows = T * ((E_total + world - 1) // world)
        padded = torch.zeros(rows, payload.shape[1])
        padded[:payload.shape[0]] = payload
        out = udist.all_gather_rows(padded)
        rec = udist.unpack_trajectory(payload)
        ok_roundtrip = (torch.equal(rec["obs"], obs.reshape(-1, 5, 14)) and
                        torch.equal(rec["actions"], actions.reshape(-1).long()) and
                        torch.equal(rec["advantages"], f[3].reshape(-1)))
        adv = f[3].reshape(-1).double()
        partials = torch.stack([adv.sum(), (adv * adv).sum()])
        mom = udist.global_moments(partials, adv.numel())
        q.put((rank, start, cnt, out.numpy(), payload.numpy(), ok_roundtrip, mom.numpy(), adv.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_and_moments(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # shards tile [0, E_total) exactly, in rank order
    starts = [r[1] for r in res]; cnts = [r[2] for r in res]
    assert starts[0] == 0 and all(starts[i] + cnts[i] == starts[i + 1] for i in range(world - 1))
    assert sum(cnts) == 10
    rows = res[0][3].shape[0] // world
    for r in res:
        assert r[5]
        for k in range(world):   # every rank sees every rank's payload at slot k
            pay = res[k][4]
            np.testing.assert_array_equal(r[3][k * rows:k * rows + pay.shape[0]], pay)
    # global moments equal the moments of the union of all ranks' advantages
    allv = np.concatenate([r[7] for r in res])
    for r in res:
        np.testing.assert_allclose(r[6], [allv.sum(), (allv * allv).sum(), allv.size], rtol=1e-12)


def test_shard_covers_all():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "target-allocation-ppo-transformer_amd"))
    from uavhip.dist import shard
    for total in (1, 7, 4096, 32768):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = shard(total, world, r)
                seen.extend(range(s, s + c))
            assert seen == list(range(total))
