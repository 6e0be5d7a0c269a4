"""Multi-GPU driver above the C ABI: one process per GPU, contiguous clip shards, one all-gather.

SURVEY.md 8(e): clips are independent (frozen BatchNorm statistics, no cross-clip state), so the
batch shards with no data-path collective.  Rank r owns clips [r*n/W, (r+1)*n/W); after its shard
runs through the fused pipeline the per-shard class probabilities are all-gathered (RCCL over xGMI
with the 'nccl' backend on ROCm; gloo in the CPU tests) so every rank holds the full [n, K] result,
in clip order.
"""
import torch
import torch.distributed as dist


def shard_range(n_total, rank, world):
    """Contiguous [lo, hi) of clips owned by `rank` (the first n % world ranks get one extra)."""
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_logits(local, n_total=None, out=None):
    """All-gather per-shard [n_r, K] tensors into the full [n, K] in rank order.

    With ``n_total`` the shard sizes follow ``shard_range`` and need no exchange (the per-step path
    of bench.py); without it they are all-gathered first.  Equal shards use one
    ``all_gather_into_tensor`` (into ``out`` when given, e.g. a buffer reused across steps); ragged
    shards pad to the largest and trim."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world == 1:
        if out is not None:
            out.copy_(local)
            return out
        return local
    if n_total is not None:
        all_sizes = [hi - lo for lo, hi in (shard_range(n_total, r, world) for r in range(world))]
        if all_sizes[dist.get_rank()] != local.shape[0]:
            raise ValueError(f'rank {dist.get_rank()} holds {local.shape[0]} rows, shard_range says '
                             f'{all_sizes[dist.get_rank()]} of {n_total}')
    else:
        sizes = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
        all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
        dist.all_gather(all_sizes, sizes)
        all_sizes = [int(s.item()) for s in all_sizes]
    m = max(all_sizes)
    if all(s == m for s in all_sizes):
        if out is None:
            out = torch.empty((world * m,) + tuple(local.shape[1:]), dtype=local.dtype,
                              device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous())
        return out
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    full = torch.cat([p[:s] for p, s in zip(parts, all_sizes)])
    if out is not None:
        out.copy_(full)
        return out
    return full


def sharded_predict(pcm_all, model_kind, ctx, rank, world, on_device=None):
    """Host-side convenience: run this rank's shard of `pcm_all` (numpy int16 [n, L]) through the
    fused pipeline on `ctx` and return the gathered probabilities [n, K] (torch).  The gather
    runs on ctx's device (RCCL) unless the process group is gloo (or on_device=False): then on the
    host."""
    import numpy as np
    lo, hi = shard_range(len(pcm_all), rank, world)
    shard = np.ascontiguousarray(pcm_all[lo:hi])
    if model_kind == 0:
        probs, _, _ = ctx.od_pipeline(shard)
    else:
        probs, _, _ = ctx.si_pipeline(shard)
    if on_device is None:
        on_device = dist.is_initialized() and dist.get_backend() != 'gloo'
    t = torch.from_numpy(probs)
    if on_device:
        t = t.to(f'cuda:{ctx.device}')
    return gather_logits(t, len(pcm_all))
