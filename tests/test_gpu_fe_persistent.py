"""The persistent OD front-end at the benchmarked batch sizes.

`od_fe3_kernel` launches min(n, #CU) workgroups; workgroup b handles clips b, b + G, b + 2G, ...
(G = grid size) and finishes clip c's epilogue (norm / dB / image stores) inside the next clip's
first tile.  That carry path only runs when a workgroup owns more than one clip, i.e. n > #CU -- the
config-2 batch of 4 096 clips gives every workgroup 16.  These tests run 4 096 and 4 096 + 37 clips
with ragged lengths and check
  * every output of every clip bit for bit against calls of at most #CU clips (one clip per
    workgroup: no carry), and sampled clips against batch-1 calls;
  * the oracle (norm <= 1e-4, dB <= 5e-3, exact ZCR counts, image <= 1 LSB) on the clips that
    workgroups process first, in the middle and last;
  * the same through the float-PCM entry (mmla_od_features_f32) at 300+ clips.
Reference: OverlapDetection/scripts/overlap_features_generator.py:65-151.
"""
import numpy as np
import pytest

from oracle import compare, od_fe

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from mmla_audio_amd import _lib
    return _lib.Context(0)


@pytest.fixture(scope='module')
def n_cu():
    import torch
    return torch.cuda.get_device_properties(0).multi_processor_count


def _clips(n, seed):
    """n synthetic 2.5 s clips (the bench's five classes, made on the GPU) + ragged lengths: a
    quarter of the clips get a random length in [0, 40 000], a few the edge lengths"""
    from mmla_audio_amd.synthetic import make_clips
    pcm = make_clips(n, 40000, seed=seed).cpu().numpy()
    rng = np.random.default_rng(seed)
    lens = np.full(n, 40000, np.int32)
    pick = rng.random(n) < 0.25
    lens[pick] = rng.integers(0, 40001, size=int(pick.sum()))
    edge = [0, 1, 399, 400, 23999, 24000, 24001]
    lens[rng.choice(n, len(edge), replace=False)] = edge
    for i in range(n):      # samples past a clip's length are garbage the kernel must not read
        pcm[i, lens[i]:] = 12345
    return pcm, lens


def _equal(a, b):
    return np.array_equal(a, b, equal_nan=True)


def _chunked(call, pcm, lens, step):
    parts = [call(pcm[c:c + step], lens[c:c + step]) for c in range(0, len(pcm), step)]
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


def _sample(n, grid):
    """clips that workgroups run first (c < G), in the middle and last (c >= n - G), spread over
    workgroups with more and fewer clips"""
    per = -(-n // grid)
    idx = {0, 1, grid - 1, n - 1, n - 2, n - grid}
    for b in (0, 5, (n - 1) % grid, grid // 2, grid - 1):
        owned = list(range(b, n, grid))
        idx.update((owned[0], owned[len(owned) // 2], owned[-1]))
    assert per > 1
    return sorted(i for i in idx if 0 <= i < n)


def _check_batch(ctx, n_cu, pcm, lens, f, call):
    n = len(pcm)
    grid = min(n, n_cu)
    # every clip: one-clip-per-workgroup calls give bit-identical outputs
    ref = _chunked(call, pcm, lens, grid)
    for k in f:
        assert _equal(f[k], ref[k]), f'{k}: multi-clip workgroups differ from one clip per workgroup'
    idx = _sample(n, grid)
    counts = []
    for i in idx:
        one = call(pcm[i:i + 1], lens[i:i + 1])
        for k in f:
            assert _equal(one[k][0], f[k][i]), f'clip {i} ({k}) differs from its batch-1 result'
        want = od_fe.od_features(pcm[i, :lens[i]])
        counts.append(compare.od_clip_compare(f, i, want, f'clip {i} (len {lens[i]})'))
    compare.od_lsb_budget(counts)


@pytest.mark.parametrize('n', [4096, 4096 + 37])
def test_od_features_many_clips_per_workgroup(ctx, n_cu, n):
    pcm, lens = _clips(n, seed=4100 + n)
    call = lambda p, ln: ctx.od_features(p, lens=ln)
    f = call(pcm, lens)
    _check_batch(ctx, n_cu, pcm, lens, f, call)


def test_od_features_f32_many_clips_per_workgroup(ctx, n_cu):
    """mmla_od_features_f32 (librosa.load float scale) with > 1 clip per workgroup"""
    n = max(300, n_cu + 45)
    pcm, lens = _clips(n, seed=4300)
    y = (pcm.astype(np.float32) / np.float32(32768.0)).astype(np.float32)
    y[::3] *= np.float32(0.37)          # values that are not int16-representable
    call = lambda p, ln: ctx.od_features(p, lens=ln)
    f = call(y, lens)
    assert len(pcm) > n_cu
    _check_batch(ctx, n_cu, y, lens, f, call)
    # on int16-derived samples (y = x / 32768) the float entry equals the int16 entry bit for bit
    g = ctx.od_features(pcm, lens=lens)
    keep = np.arange(n) % 3 != 0
    for k in g:
        assert _equal(g[k][keep], f[k][keep]), k
