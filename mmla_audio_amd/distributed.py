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


def gather_logits(local, n_total=None, out=None, force_collective=False):
    """All-gather per-shard [n_r, K] tensors into the full [n, K] in rank order.

    With ``n_total`` the shard sizes follow ``shard_range`` and need no exchange (the per-step path
    of bench.py); without it they are all-gathered first.  Equal shards use one
    ``all_gather_into_tensor`` (into ``out`` when given, e.g. a buffer reused across steps); ragged
    shards pad to the largest and trim.  A one-rank group returns ``local`` (copied into ``out``)
    without a collective unless ``force_collective``: the GPU test runs the RCCL calls of the
    multi-rank path at world size 1 with it (tests/test_gpu_rccl.py)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world == 1 and not (force_collective and dist.is_initialized()):
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


# ---- SI whole-conversation mode sharded by frame range ----------------------------
# speaker_identification_post_processing.py:255-272 computes MFCC + deltas over the WHOLE conversation
# and predicts its 256-frame windows in one batch.  A rank owns a contiguous range of windows; the
# frames it needs beyond them are the halo: MFCC(t) reads samples [160 t, 160 t + 400) after a
# pre-emphasis that needs sample 160 t - 1, and delta-delta(t) reads MFCC(t - 4 .. t + 4).  So the
# rank computes frames [f0 - 5, f1 + 4) from its own slice of the signal (the 5th frame before f0 only
# absorbs the slice's pre-emphasis start and the deltas' edge padding) and keeps [f0, f1): identical
# to the single-process features, with no collective before the logits gather.
SI_WIN_FRAMES, SI_HOP, SI_FRAME = 256, 160, 400
_HALO_BEFORE, _HALO_AFTER = 5, 4


def conversation_frames(n_samples):
    """psf framesig's frame count and the number of 256-frame windows of a conversation."""
    t = 1 if n_samples <= SI_FRAME else 1 + -(-(n_samples - SI_FRAME) // SI_HOP)
    return t, -(-t // SI_WIN_FRAMES)


def conversation_shard(n_samples, rank, world):
    """-> (w0, w1, s_lo, s_hi, keep): this rank's windows [w0, w1), the signal slice [s_lo, s_hi)
    it computes features on, and the first kept frame's index within that slice's frames."""
    t, s = conversation_frames(n_samples)
    w0, w1 = shard_range(s, rank, world)
    if w1 <= w0:                        # more ranks than windows: nothing to compute
        return w0, w1, 0, 0, 0
    f0, f1 = w0 * SI_WIN_FRAMES, min(w1 * SI_WIN_FRAMES, t)
    a = max(f0 - _HALO_BEFORE, 0)
    b = min(f1 + _HALO_AFTER, t)
    s_hi = n_samples if b == t else SI_HOP * (b - 1) + SI_FRAME
    return w0, w1, SI_HOP * a, s_hi, f0 - a


def conversation_features_shard(sig, rank, world, features_seq):
    """This rank's windows of the conversation's [S, 256, 39] features (float32, as the kernel
    returns them).  ``features_seq(slice) -> [S', 256, 39]`` is the whole-signal feature call
    (``Context.si_features_seq``)."""
    import numpy as np
    sig = np.ascontiguousarray(sig, dtype=np.int16).ravel()
    t, _ = conversation_frames(sig.size)
    w0, w1, s_lo, s_hi, keep = conversation_shard(sig.size, rank, world)
    out = np.zeros((w1 - w0, SI_WIN_FRAMES, 39), np.float32)
    if w1 <= w0:
        return out
    f = np.asarray(features_seq(sig[s_lo:s_hi])).reshape(-1, 39)
    n_keep = min(w1 * SI_WIN_FRAMES, t) - w0 * SI_WIN_FRAMES
    out.reshape(-1, 39)[:n_keep] = f[keep:keep + n_keep]
    return out


def sharded_conversation_predict(sig, ctx, rank, world, on_device=None):
    """post_analysing's whole-conversation predict (speaker_identification_post_processing.py:
    255-272) sharded by window range: this rank's windows through SI-NET on ctx, the logits
    all-gathered in window order -> [S, K] on every rank."""
    import numpy as np
    feat = conversation_features_shard(sig, rank, world, ctx.si_features_seq)
    if ctx.si_classes is None:
        raise RuntimeError('load the SI weights (Context.load_weights) before predicting')
    probs = ctx.si_forward(feat) if len(feat) else np.zeros((0, ctx.si_classes), np.float32)
    if on_device is None:
        on_device = dist.is_initialized() and dist.get_backend() != 'gloo'
    t = torch.from_numpy(np.ascontiguousarray(probs, dtype=np.float32))
    if on_device:
        t = t.to(f'cuda:{ctx.device}')
    _, s = conversation_frames(np.asarray(sig).size)
    return gather_logits(t, s)
