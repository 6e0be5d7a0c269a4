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


def gather_logits(local, n_total=None):
    """All-gather per-shard [n_r, K] tensors into the full [n, K] in rank order.

    Equal shards use one ``all_gather_into_tensor``; ragged shards pad to the largest and trim."""
    world = dist.get_world_size()
    if world == 1:
        return local
    sizes = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes)
    all_sizes = [int(s.item()) for s in all_sizes]
    m = max(all_sizes)
    if all(s == m for s in all_sizes):
        out = torch.empty((world * m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous())
        return out
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:s] for p, s in zip(parts, all_sizes)])


def sharded_predict(pcm_all, model_kind, ctx, rank, world, clip_len=None):
    """Host-side convenience: run this rank's shard of `pcm_all` (numpy int16 [n, L]) through the
    fused pipeline on `ctx` and return the gathered probabilities (torch, on ctx's device)."""
    import numpy as np
    lo, hi = shard_range(len(pcm_all), rank, world)
    shard = np.ascontiguousarray(pcm_all[lo:hi])
    if model_kind == 0:
        probs, _ = ctx.od_pipeline(shard)
    else:
        probs, _, _ = ctx.si_pipeline(shard)
    t = torch.from_numpy(probs).to(f'cuda:{ctx.device}' if torch.cuda.is_available() else 'cpu')
    return gather_logits(t, len(pcm_all))
