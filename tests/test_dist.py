"""Multi-process (world_size 2 and 3, gloo on CPU) checks of the data-parallel plumbing in
uavhip.dist: env sharding, the single trajectory all-gather of the compact format (rank order,
record layout; every rank's windows rebuilt exactly from its rows / done flags / first windows by
the oracle's deque restatement) and the global advantage moments all-reduce. The RCCL path runs
the same functions with backend "nccl"; the GPU rebuild kernel is checked in test_gpu_policy_gae."""
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


def _deque_windows(T, E, g):
    """Windows as UAVEnv's deque produces them (zeros after a reset, shift + append per step),
    T + 1 steps (the rollout buffer keeps the next window), with random rows and done flags."""
    dones = (torch.rand(T, E, generator=g) < 0.25).to(torch.uint8)
    obs = torch.zeros(T + 1, E, 5, 14)
    w = torch.randn(E, 5, 14, generator=g)
    w[: E // 2, :2] = 0  # some envs mid-way through their first 5 steps
    for t in range(T + 1):
        if t > 0:
            nxt = torch.zeros_like(w)
            for e in range(E):
                if not dones[t - 1, e]:
                    nxt[e, :4] = w[e, 1:]
            nxt[:, 4] = torch.randn(E, 14, generator=g)
            w = nxt
        obs[t] = w
    return obs, dones


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
        E = (E_total + world - 1) // world  # equal payloads per rank (the last shard padded)
        g = torch.Generator().manual_seed(1000 + rank)
        obs, dones = _deque_windows(T, E, g)
        actions = torch.randint(0, 2, (T, E), generator=g, dtype=torch.int8)
        f = [torch.randn(T, E, generator=g) for _ in range(4)]
        payload = udist.pack_compact(obs, actions, f[0], f[1], f[2], f[3], dones)
        assert payload.numel() == udist.compact_floats(T, E)
        out = udist.all_gather_rows(payload.view(1, -1))
        adv = f[3][:, :cnt].reshape(-1).double()
        partials = torch.stack([adv.sum(), (adv * adv).sum()])
        mom = udist.global_moments(partials, adv.numel())
        q.put((rank, start, cnt, out.numpy(), payload.numpy(), obs.numpy(), dones.numpy(), mom.numpy(), adv.numpy()))
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
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle.windows import windows_from_rows
    T, E = 6, res[0][5].shape[1]
    for r in res:
        gathered = r[3]
        assert gathered.shape == (world, res[0][4].size)
        for k in range(world):   # every rank sees every rank's payload at slot k
            np.testing.assert_array_equal(gathered[k], res[k][4])
            # the compact record rebuilds rank k's windows exactly (deque semantics)
            nr, ns = T * E * 14, T * E * 6
            rows = gathered[k][:nr].reshape(T, E, 14)
            scal = gathered[k][nr:nr + ns].reshape(T, E, 6)
            first = gathered[k][nr + ns:].reshape(E, 5, 14)
            np.testing.assert_array_equal(windows_from_rows(first, rows, scal[..., 5]), res[k][5][:T])
            np.testing.assert_array_equal(scal[..., 5], res[k][6])
    # global moments equal the moments of the union of all ranks' advantages
    allv = np.concatenate([r[8] for r in res])
    for r in res:
        np.testing.assert_allclose(r[7], [allv.sum(), (allv * allv).sum(), allv.size], rtol=1e-12)


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


def _shard_worker(rank, world, port, q, bases):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "target-allocation-ppo-transformer_amd"))
    import torch.distributed as dist
    from uavhip.dist import resolve_shards, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        start, cnt = shard(10, world, rank)
        out["default"] = resolve_shards(cnt, start)                   # total = sum of the ranks' E
        out["explicit"] = resolve_shards(cnt, start, total_envs=10)
        for key, base, total in (("same_base", 0, None), ("bad_total", start, 12), ("custom", bases[rank], None)):
            try:
                out[key] = resolve_shards(cnt, base, total_envs=total)
            except ValueError as exc:
                out[key] = "ValueError: " + str(exc)
        # a sub-group (RolloutEngine(group=...)): only its ranks take part, the total is theirs
        sub = dist.new_group([0, 1])  # collective over the world
        if rank < 2:
            out["subgroup"] = resolve_shards(4, 4 * rank, group=sub)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_resolve_shards_checks_the_rank_blocks():
    """RolloutEngine's total_envs (the sampling counters t * total + env_base + e and the global
    advantage count T * total, ppo.py:94) comes from all-gathering the ranks' (E, env_base): the
    sum by default; overlapping blocks (every rank left at env_base 0) or a total that is not the sum
    raise on every rank instead of sampling duplicate actions / normalising with a wrong count."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    bases = [6, 0, 3]  # disjoint blocks in another rank order: rank 0 [6, 10), rank 1 [0, 3), rank 2 [3, 6)
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q, bases)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        out = res[r]
        assert out["default"] == out["explicit"] == 10
        assert str(out["same_base"]).startswith("ValueError") and "disjoint" in out["same_base"]
        assert str(out["bad_total"]).startswith("ValueError")
        assert out["custom"] == 10  # disjoint blocks in any rank order are fine
        if r < 2:
            assert out["subgroup"] == 8  # the sub-group's two blocks, not the world's


def test_resolve_shards_single_process():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "target-allocation-ppo-transformer_amd"))
    from uavhip.dist import resolve_shards
    assert resolve_shards(7, 0) == 7
    assert resolve_shards(7, 3, total_envs=10) == 10
    with pytest.raises(ValueError):
        resolve_shards(7, 4, total_envs=10)


class _FakeMapper:
    """CPU stand-in for uavhip.dist.HipPeerMapper: device `dev`, allocation failing when asked to,
    peer access from this device to the devices in `no_peer` refused."""

    def __init__(self, dev, fail_alloc=False, no_peer=()):
        self.dev, self.fail_alloc, self.no_peer = dev, fail_alloc, set(no_peer)
        self.opened, self.closed = [], []

    def identity(self):
        return self.dev

    def alloc(self, shape):
        if self.fail_alloc:
            raise RuntimeError("out of memory (simulated)")
        return torch.zeros(*shape)

    def sync(self):
        pass

    def export(self, t):
        return (b"h" * 64, 0)

    def can_access(self, peer):
        return peer == self.dev or peer not in self.no_peer

    def open(self, handle):
        self.opened.append(handle)
        return (len(self.opened), 0)

    def close(self, m):
        self.closed.append(m)


def _ipc_setup_worker(rank, world, port, q, case):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "target-allocation-ppo-transformer_amd"))
    import torch.distributed as dist
    from uavhip.dist import IpcAllGather
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if case == "alloc":      # rank 1 cannot allocate its buffers
            m = _FakeMapper(rank, fail_alloc=rank == 1)
        elif case == "peer":     # rank 2's device has no peer access to rank 0's
            m = _FakeMapper(rank, no_peer=(0,) if rank == 2 else ())
        else:                    # every pair has peer access (one device per rank)
            m = _FakeMapper(rank)
        try:
            x = IpcAllGather(16, torch.device("cpu"), None, mapper=m)
            q.put((rank, ("ok", sorted(x.peer_send), x.peer_devices, len(m.opened))))
        except RuntimeError as exc:
            q.put((rank, ("error", str(exc), len(m.opened), len(m.closed))))
    finally:
        dist.destroy_process_group()


def _run_ipc_case(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ipc_setup_worker, args=(r, world, port, q, case)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_ipc_exchange_setup_fails_on_every_rank_together():
    """bench.py's pipelined exchange falls back to RCCL's all-gather when any rank cannot set it up:
    IpcAllGather's setup is collective, so a failure on one rank raises on every rank (none is left
    waiting in a collective the failed rank skipped)."""
    res = _run_ipc_case(2, "alloc")
    assert res[1][0] == "error" and "this rank" in res[1][1], res
    assert res[0][0] == "error" and "another rank" in res[0][1], res


def test_ipc_exchange_peer_access_decision():
    """Peer access is checked for every (this device, peer device) pair before anything is mapped
    (HipPeerMapper.can_access: hipDeviceCanAccessPeer + hipDeviceEnablePeerAccess). One pair
    without it (rank 2's device cannot reach rank 0's) makes EVERY rank raise -- so every rank falls
    back to RCCL together -- and the ranks that had mapped peer buffers unmap them; with every pair
    reachable each rank maps its world - 1 peers' two send buffers and learns their devices."""
    world = 3
    res = _run_ipc_case(world, "peer")
    for r in range(world):
        assert res[r][0] == "error", res
        assert ("this rank" if r == 2 else "another rank") in res[r][1], res
        assert "no peer access" in res[r][1], res
        assert res[r][2] == res[r][3]  # whatever was mapped was unmapped
    res = _run_ipc_case(world, "all")
    for r in range(world):
        status, peers, devs, opened = res[r]
        assert status == "ok" and peers == [j for j in range(world) if j != r], res
        assert devs == {j: j for j in range(world)} and opened == 2 * (world - 1)


def _capture_vote_worker(rank, world, port, q):
    import sys
    import types
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "target-allocation-ppo-transformer_amd"))
    import torch.distributed as dist
    from uavhip.train import FusedPPOTrainer
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class _Trainer(FusedPPOTrainer):
        """The data-parallel capture / run logic without a GPU: the capture fails on rank 1, an
        eager step only counts."""
        captures = 0
        eager = 0

        def _capture_graph(self, steps):
            self.captures += 1
            if self.rank == 1:
                raise RuntimeError("simulated capture failure")
            return object()

        def _eager_step(self, perm, b):
            self.eager += 1
            self.stats[3] += 1

    try:
        tr = _Trainer.__new__(_Trainer)
        tr.world, tr.rank, tr.dp, tr.graph_collectives = world, rank, True, True
        tr.allreduce = lambda t: dist.all_reduce(t)
        tr.device, tr.global_minibatch, tr.minibatch, tr.n, tr.n_local = torch.device("cpu"), 128, 64, 3 * 128, None
        tr.graphs, tr.capture_failed = {}, {}
        tr.perm, tr.stats = torch.zeros(3 * 128, dtype=torch.int32), torch.zeros(4, dtype=torch.float64)
        tr.policy = types.SimpleNamespace()
        res = []
        for _ in range(2):  # the second run must not capture (nor vote) again
            out = tr.run(epochs=2, generator=torch.Generator().manual_seed(1), use_graph=True)
            res.append(out[3])
        q.put((rank, (tr.captures, tr.eager, res, dict(tr.capture_failed), tr.graph is None)))
    finally:
        dist.destroy_process_group()


def test_data_parallel_capture_failure_is_voted_and_remembered():
    """FusedPPOTrainer.capture on a data-parallel group: a capture that fails on one rank makes every
    rank drop its graph (the ranks vote with an all-reduce), each rank keeps why (the failing rank its
    exception, the others the vote) per step count, and later run()s step eagerly without capturing
    or voting again -- so no rank replays a graph whose collectives the others never join."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_capture_vote_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        captures, eager, counts, failed, no_graph = res[r]
        assert captures == 1, res            # one capture attempt, then remembered
        assert eager == 2 * 2 * 3 and counts == [6, 6], res  # 2 runs x 2 epochs x 3 steps, all eager
        assert no_graph and list(failed) == [3], res
        assert ("simulated capture failure" if r == 1 else "other rank") in failed[3], res
