"""Data-parallel plumbing for the rollout: one process per GPU, envs sharded across
ranks (independent episodes, no cross-env term in UAVEnv.step), and ONE exchange per PPO
iteration -- an all-gather of the trajectory records over RCCL (backend "nccl" on ROCm) -- plus a
3-double all-reduce so every rank normalises advantages with the statistics of the whole batch
(ppo.py:94 normalises over the full buffer).
"""
import torch
import torch.distributed as dist

# Compact exchange format (one flat fp32 payload per rank): the row each step pushes into the
# observation window ([T][E][14], = window slot 4), the per-transition scalars ([T][E][6]: action,
# logp, value, return, advantage, done) and the window at step 0 ([E][70]). A window is the last 5
# rows of its episode (zeros before the episode's first step), so the receivers rebuild all T
# windows on the GPU (uavhip_windows_from_rows): 20 floats per transition instead of 76.
ROW_FLOATS = 14
SCALARS = ("actions", "logp", "values", "returns", "advantages", "dones")


def shard(total, world, rank):
    """Contiguous env shard [start, start + count) of `total` envs for `rank`."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def resolve_shards(E, env_base, total_envs=None, group=None, device=None):
    """Total env count of a data-parallel rollout, checked across the ranks (once, at engine setup).

    Every rank's env block [env_base, env_base + E) must be disjoint from the others' and inside
    [0, total): the sampling counters t * total + env_base + e (RolloutEngine) are then unique over
    the ranks, and T * total is the element count of the global advantage moments (ppo.py:94). With
    torch.distributed initialised (world > 1) the blocks are all-gathered and total defaults to the
    sum of every rank's E; a mismatch (e.g. every rank left at env_base 0) raises instead of sampling
    duplicate actions or normalising with a wrong count. One process: total_envs or E.
    Collective over `group` (every rank of it must call it); on an RCCL group the exchanged tensor
    lives on `device` (the env's device; default the current device)."""
    E, env_base = int(E), int(env_base)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        total = E if total_envs is None else int(total_envs)
        if env_base < 0 or env_base + E > total:
            raise ValueError(f"env block [{env_base}, {env_base + E}) outside total_envs {total}")
        return total
    world = dist.get_world_size(group)
    dev = "cpu" if dist.get_backend(group) == "gloo" else (
        torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device()))
    mine = torch.tensor([[E, env_base]], dtype=torch.int64, device=dev)
    blocks = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(blocks, mine, group=group)
    blocks = sorted(tuple(int(v) for v in b.view(-1).tolist()) for b in blocks)  # (E, base) per rank
    total_sum = sum(b[0] for b in blocks)
    total = total_sum if total_envs is None else int(total_envs)
    spans = sorted((base, base + e) for e, base in blocks)
    overlap = any(spans[i][1] > spans[i + 1][0] for i in range(len(spans) - 1))
    if overlap or spans[0][0] < 0 or spans[-1][1] > total or total != total_sum:
        raise ValueError(f"data-parallel env blocks {spans} (E, env_base per rank) must be disjoint and tile "
                         f"total_envs {total} = sum of E {total_sum}: build each rank's VecUAVEnv with "
                         f"env_base = its shard start (uavhip.dist.shard)")
    return total


def compact_floats(T, E):
    """Floats of one rank's payload."""
    return T * E * (ROW_FLOATS + len(SCALARS)) + E * 70


def pack_compact(obs, actions, logp, values, returns, advantages, dones):
    """obs [>=T, E, 5, 14] policy inputs and [T, E] per-step tensors -> flat fp32 payload."""
    T, E = actions.shape[:2]
    rows = obs[:T, :, 4, :].reshape(-1)
    scal = torch.stack([actions.float(), logp.float(), values.float(), returns.float(), advantages.float(),
                        dones.float()], dim=-1).reshape(-1)
    return torch.cat([rows.float(), scal, obs[0].reshape(-1).float()]).contiguous()


def unpack_compact(payloads, T, E, copy=False):
    """[world, compact_floats] gathered payloads -> dict of [world * T * E, ...] tensors in (rank,
    step, env) order; obs rebuilt on the GPU (uavhip_windows_from_rows; the HIP library is
    required -- there is no host fallback). The scalar columns are views into `payloads` unless
    copy=True (a receive buffer that is rewritten later: IpcAllGather's)."""
    from ._lib import LIB, check, ptr, stream_handle
    world = payloads.shape[0]
    F = compact_floats(T, E)
    if payloads.shape[1] != F or payloads.dtype != torch.float32 or not payloads.is_contiguous():
        raise ValueError("payloads must be a contiguous fp32 [world, compact_floats(T, E)] tensor")
    nr = T * E * ROW_FLOATS
    ns = T * E * len(SCALARS)
    scal = payloads[:, nr:nr + ns].reshape(world * T * E, len(SCALARS))
    if copy:
        scal = scal.clone()
    obs = torch.empty(world * T * E, 5, 14, dtype=torch.float32, device=payloads.device)
    base = payloads.data_ptr()
    check(LIB.uavhip_windows_from_rows(base + 4 * (nr + ns), base, base + 4 * (nr + len(SCALARS) - 1),
                                       len(SCALARS), F, world, T, E, ptr(obs), stream_handle()),
          "uavhip_windows_from_rows")
    out = {k: scal[:, i] for i, k in enumerate(SCALARS)}
    out["actions"] = out["actions"].to(torch.int8)
    out["obs"] = obs
    return out


def all_gather_rows(payload, group=None):
    """Concatenate every rank's [rows, F] payload in rank order (equal rows per rank); one
    all_gather_into_tensor over RCCL."""
    world = dist.get_world_size(group)
    if world == 1:
        return payload
    out = torch.empty(world * payload.shape[0], *payload.shape[1:], dtype=payload.dtype, device=payload.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, payload, group=group)
    else:
        dist.all_gather(list(out.chunk(world)), payload, group=group)
    return out


def global_moments(partials, count, group=None):
    """Fold this rank's fp64 (sum, sum of squares) block partials and all-reduce them with the
    element count -> tensor [S, S2, n] (fp64) describing the whole data-parallel batch."""
    p = partials.view(-1, 2).sum(0)
    t = torch.cat([p, torch.tensor([float(count)], dtype=torch.float64, device=p.device)])
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, group=group)
    return t


def normalize_global(adv, moments, count=None):
    """adv <- (adv - mean) / (std + 1e-7) with the global moments, on the GPU kernel. count: the
    global element count when the caller knows it (else read back from moments: a host sync)."""
    from ._lib import LIB, check, ptr, stream_handle
    m = moments[:2].contiguous()
    n = int(moments[2].item()) if count is None else int(count)
    check(LIB.uavhip_adv_normalize(ptr(adv), adv.numel(), ptr(m), 1, n, None, stream_handle()),
          "uavhip_adv_normalize")
    return adv


class HipPeerMapper:
    """The device side of IpcAllGather over the C ABI (include/uavhip.h, N > 1 exchange): export a
    send buffer as an IPC handle, check / enable peer access to another device, map a peer's buffer
    into THIS device's address space (hipIpcOpenMemHandle from the current device: no HIP context
    is created on the exporter's device) and copy out of it on a stream of this device."""

    def __init__(self, device):
        self.device = torch.device(device)
        self._maps = {}  # handle bytes -> [base pointer, references]: two buffers of one allocation map once

    def device_index(self):
        return self.device.index if self.device.index is not None else torch.cuda.current_device()

    def identity(self):
        """This rank's device as the ranks can compare it: its PCI bus id (ordinals are local to a
        process -- ranks started with their own HIP_VISIBLE_DEVICES all see device 0)."""
        import ctypes
        from ._lib import LIB, check
        buf = ctypes.create_string_buffer(64)
        check(LIB.uavhip_device_pci_id(int(self.device_index()), buf, 64), "uavhip_device_pci_id")
        return buf.value.decode().lower()

    def alloc(self, shape):
        return torch.zeros(*shape, dtype=torch.float32, device=self.device)

    def sync(self):
        torch.cuda.synchronize(self.device)

    def export(self, t):
        import ctypes
        from ._lib import LIB, check
        h = (ctypes.c_char * 64)()
        off = ctypes.c_uint64(0)
        check(LIB.uavhip_ipc_export(t.data_ptr(), h, ctypes.byref(off)), "uavhip_ipc_export")
        return bytes(h), int(off.value)

    def can_access(self, peer):
        """Peer access from this rank's device to the device a peer published as identity(): the
        same bus id is the same device; otherwise the bus id is mapped to this process's ordinal
        (not visible here -> no access) and hipDeviceCanAccessPeer / hipDeviceEnablePeerAccess ask."""
        import ctypes
        from ._lib import LIB, check
        if peer == self.identity():
            return True
        local = ctypes.c_int32(-1)
        check(LIB.uavhip_device_from_pci_id(str(peer).encode(), ctypes.byref(local)), "uavhip_device_from_pci_id")
        if local.value < 0:
            return False
        ok = ctypes.c_int32(0)
        with torch.cuda.device(self.device):
            check(LIB.uavhip_peer_access(int(local.value), ctypes.byref(ok)), "uavhip_peer_access")
        return bool(ok.value)

    def open(self, handle):
        import ctypes
        from ._lib import LIB, check
        h, off = handle
        if h not in self._maps:
            p = ctypes.c_void_p(0)
            with torch.cuda.device(self.device):
                check(LIB.uavhip_ipc_open(h, 0, ctypes.byref(p)), "uavhip_ipc_open")
            self._maps[h] = [int(p.value), 0]
        self._maps[h][1] += 1
        return (self._maps[h][0] + off, h)

    def close(self, mapped):
        from ._lib import LIB
        ent = self._maps.get(mapped[1])
        if ent is None:
            return
        ent[1] -= 1
        if ent[1] == 0:
            with torch.cuda.device(self.device):
                LIB.uavhip_ipc_close(ent[0])
            del self._maps[mapped[1]]

    def copy(self, dst, mapped, stream):
        """dst (a tensor of this device) <- the mapped peer buffer, on `stream`."""
        from ._lib import LIB, check
        check(LIB.uavhip_copy_async(dst.data_ptr(), mapped[0], dst.numel() * dst.element_size(),
                                    stream.cuda_stream), "uavhip_copy_async")


class IpcAllGather:
    """The trajectory all-gather as peer-to-peer copies out of IPC-mapped buffers, pipelined one
    iteration behind the rollout so that iteration k's exchange runs beside iteration k + 1's
    rollout: RCCL's all-gather kernels cannot become resident beside k_rollout_steps,
    which holds every CU, while a device-to-device copy between two GPUs is a DMA transfer.

    Every rank owns two send buffers (iteration parity p) that the other ranks map through IPC
    (handles exchanged over `group`, a gloo group) and two receive buffers [world, floats]. Setup
    checks peer access from this rank's device to every other rank's device (hipDeviceCanAccessPeer,
    then hipDeviceEnablePeerAccess) and maps each peer buffer into this device's own address space
    (no HIP context on any other device). submit(payload) enqueues the copy of this iteration's
    payload into send[p] on the current stream. progress() completes the pending exchange: the host
    waits until its payload is written and its copies of the previous iteration are done, a host
    barrier (every rank: both), then the side stream -- a stream of this rank's device -- copies every
    peer's send[p] into recv[p] (and its own). Send buffers are rewritten only after every rank passed
    the barrier that follows the copies reading them, so no interprocess events are needed. Call
    progress() after enqueueing the next iteration's work: the host wait returns as that work
    starts, and the copies run beside it.

    `mapper` supplies the device operations (default HipPeerMapper; the CPU tests inject fakes)."""

    def __init__(self, floats, device, group, mapper=None):
        """Collective over `group`: every rank takes part in the same calls whether or not its own
        setup fails, and all of them raise if any rank's did (allocation, export, a pair of devices
        without peer access, or a mapping that fails) -- bench.py then falls back to RCCL's
        all-gather on every rank."""
        self.world, self.rank, self.group = dist.get_world_size(group), dist.get_rank(group), group
        self.floats, self.device = int(floats), device
        self.mapper = mapper if mapper is not None else HipPeerMapper(device)
        err, mine = None, None
        try:
            self.send = [self.mapper.alloc((self.floats,)) for _ in range(2)]
            self.recv = [self.mapper.alloc((self.world, self.floats)) for _ in range(2)]
            self.mapper.sync()
            mine = (self.mapper.identity(), [self.mapper.export(t) for t in self.send])
        except Exception as exc:  # noqa: BLE001 -- reported collectively below
            err = exc
        objs = [None] * self.world
        dist.all_gather_object(objs, mine, group=group)
        if err is None and any(o is None for o in objs):
            err = RuntimeError("another rank could not export its buffers")
        self.peer_devices = {j: o[0] for j, o in enumerate(objs) if o is not None}
        self.peer_send = {}
        if err is None:
            try:
                no_peer = [j for j, o in enumerate(objs) if j != self.rank and not self.mapper.can_access(o[0])]
                if no_peer:
                    raise RuntimeError(f"no peer access from device {mine[0]} to the devices of ranks {no_peer} "
                                       f"({[objs[j][0] for j in no_peer]})")
                self.peer_send = {j: [self.mapper.open(h) for h in o[1]] for j, o in enumerate(objs) if j != self.rank}
            except Exception as exc:  # noqa: BLE001
                err = exc
        oks = [None] * self.world
        dist.all_gather_object(oks, None if err is None else repr(err), group=group)
        bad = {j: e for j, e in enumerate(oks) if e is not None}
        if bad:
            self.close()
            raise RuntimeError(f"IpcAllGather setup failed on {'this' if err else 'another'} rank: "
                               f"{ {j: e for j, e in bad.items()} }")
        self.side = torch.cuda.Stream(device) if self.device.type == "cuda" else None
        self.packed = [torch.cuda.Event(), torch.cuda.Event()] if self.side is not None else [None, None]
        self.copied = [None, None]
        self.k = 0
        self.pending = None
        dist.barrier(group=group)

    def close(self):
        """Unmap the peers' buffers (collective use: after the last progress())."""
        for bufs in getattr(self, "peer_send", {}).values():
            for m in bufs:
                try:
                    self.mapper.close(m)
                except Exception:  # noqa: BLE001 -- teardown
                    pass
        self.peer_send = {}

    def submit(self, payload):
        """Enqueue this iteration's flat fp32 payload (current stream); progress() exchanges it."""
        if self.pending is not None:
            raise RuntimeError("IpcAllGather.submit: the previous payload was not progressed")
        p = self.k & 1
        self.send[p].copy_(payload.view(-1))
        self.packed[p].record()
        self.pending = p
        self.k += 1

    def progress(self):
        """Exchange the pending payload -> (receive buffer [world, floats], event recorded on the side
        stream once it is complete; the caller's stream must wait on it before reading)."""
        p = self.pending
        if p is None:
            raise RuntimeError("IpcAllGather.progress: nothing submitted")
        self.packed[p].synchronize()
        if self.copied[p ^ 1] is not None:
            self.copied[p ^ 1].synchronize()  # this rank's reads of the peers' other-parity buffers
        dist.barrier(group=self.group)
        self.side.wait_event(self.packed[p])
        with torch.cuda.stream(self.side):
            self.recv[p][self.rank].copy_(self.send[p])
            for j in sorted(self.peer_send):  # every copy on the side stream of THIS device
                self.mapper.copy(self.recv[p][j], self.peer_send[j][p], self.side)
        ev = torch.cuda.Event()
        ev.record(self.side)
        self.copied[p] = ev
        self.pending = None
        return self.recv[p], ev
