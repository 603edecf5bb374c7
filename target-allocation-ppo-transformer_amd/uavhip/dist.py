"""Data-parallel plumbing for the rollout: one process per GPU, envs sharded across
ranks (independent episodes, no cross-env term in UAVEnv.step), and ONE exchange per PPO
iteration -- an all-gather of the trajectory records over RCCL (backend "nccl" on ROCm) -- plus a
3-double all-reduce so every rank normalises advantages with the statistics of the whole batch
(ppo.py:94 normalises over the full buffer).
"""
import torch
import torch.distributed as dist

# per-transition record: 70 window floats + action, logp, value, return, advantage, reward, done
RECORD_FLOATS = 70 + 7


def shard(total, world, rank):
    """Contiguous env shard [start, start + count) of `total` envs for `rank`."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def pack_trajectory(obs, actions, logp, values, returns, advantages, rewards, dones):
    """[T, E, ...] buffers -> one fp32 [T*E, RECORD_FLOATS] payload (single collective)."""
    T, E = actions.shape[:2]
    n = T * E
    return torch.cat([obs.reshape(n, -1).float(), actions.reshape(n, 1).float(), logp.reshape(n, 1).float(),
                      values.reshape(n, 1).float(), returns.reshape(n, 1).float(), advantages.reshape(n, 1).float(),
                      rewards.reshape(n, 1).float(), dones.reshape(n, 1).float()], dim=1).contiguous()


def unpack_trajectory(payload):
    o = payload
    return dict(obs=o[:, :70].reshape(-1, 5, 14), actions=o[:, 70].long(), logp=o[:, 71], values=o[:, 72],
                returns=o[:, 73], advantages=o[:, 74], rewards=o[:, 75], dones=o[:, 76])


def all_gather_rows(payload, group=None):
    """Concatenate every rank's [rows, F] payload in rank order (equal rows per rank)."""
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


def normalize_global(adv, moments):
    """adv <- (adv - mean) / (std + 1e-7) with the global moments, on the GPU kernel."""
    from ._lib import LIB, check, ptr, stream_handle
    m = moments[:2].contiguous()
    check(LIB.uavhip_adv_normalize(ptr(adv), adv.numel(), ptr(m), 1, int(moments[2].item()), None,
                                   stream_handle()), "uavhip_adv_normalize")
    return adv
