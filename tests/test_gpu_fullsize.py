"""Full-size batches (BASELINE configs 3 and 4): every sampled clip of a 65 573-clip OD run (config
3's 65 536 clips + a partial micro-batch; exact f32: two micro-batches + 37) and a 65 536-clip SI run
equals its batch-1 result, clips are compared at every micro-batch edge (the
OD activation buffers exceed 2^31 elements there, so a 32-bit index anywhere would show), and a
sample matches the oracle to |log p - log p_ref| <= 1e-4 with identical argmax (oracle/compare.py).

Inputs are generated in HBM (mmla_audio_amd.synthetic.make_clips) and run through the
device-pointer ABI like bench.py; the batch-1 references go through the host-pointer ABI.
"""
import numpy as np
import pytest

from oracle import compare, nets, od_fe, si_fe

pytestmark = pytest.mark.gpu


def _sample(n, mb, k_random, seed):
    """first and last clip of every micro-batch + k random clips"""
    idx = set()
    for c0 in range(0, n, mb):
        idx.update((c0, min(c0 + mb, n) - 1))
    idx.update(np.random.default_rng(seed).choice(n, k_random, replace=False).tolist())
    return sorted(idx)


@pytest.mark.parametrize('prec', ['f16x3', 'f32'])
def test_od_two_microbatches(prec):
    import torch
    from mmla_audio_amd import _lib, weights
    from mmla_audio_amd.synthetic import make_clips
    c = _lib.Context(0)
    W = weights.synthetic(weights.OD, seed=77)
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    c.set_precision(_lib.PREC_F16X3 if prec == 'f16x3' else _lib.PREC_F32)
    mb = c.get_microbatch()[0]
    # config 3 (65 536 clips) and a partial micro-batch after it; exact f32: two + a partial third
    n = max(65536, 4 * mb) + 37 if prec == 'f16x3' else 2 * mb + 37
    pcm = make_clips(n, 40000, start_index=50000)
    probs = torch.empty((n, 2), dtype=torch.float32, device='cuda')
    am = torch.empty(n, dtype=torch.int32, device='cuda')
    c.od_pipeline_dev(pcm.data_ptr(), n, 40000, 40000, probs.data_ptr(), am.data_ptr())
    c.synchronize()
    idx = _sample(n, mb, 32, 1)
    sub = pcm[idx].cpu().numpy()
    probs, am = probs.cpu().numpy(), am.cpu().numpy()
    c.release_workspace()
    for j, i in enumerate(idx):
        p1, a1, _ = c.od_pipeline(sub[j:j + 1])
        assert np.array_equal(p1[0], probs[i]) and a1[0] == am[i], f'clip {i} of {n} (mb {mb})'
    if prec == 'f32':
        return
    # the network on the kernel's own image: log-probabilities to 1e-4; the argmax on the oracle
    # front-end's image (which may differ by 1 LSB on a few pixels) except at log-margin near-ties
    pick = idx[::max(1, len(idx) // 10)]
    rows = [idx.index(i) for i in pick]
    img = c.od_features(sub[rows], db=False, norm=False, zcr=False)['img'].astype(np.float32)
    err = compare.logp_err(probs[pick], nets.od_forward(img, W))
    assert err <= compare.LOGP_TOL, err
    ref = nets.od_forward(np.stack([od_fe.od_features(sub[r])['png_rgb'] for r in rows]).astype(np.float32), W)
    assert compare.argmax_ok(probs[pick], ref)


def test_si_65536_clips():
    import torch
    from mmla_audio_amd import _lib, weights
    from mmla_audio_amd.synthetic import make_clips
    c = _lib.Context(0)
    W = weights.synthetic(weights.SI, seed=78, n_classes=630)
    c.load_weights(weights.SI, weights.pack(weights.SI, W, 630), 630, _lib.HEAD_SOFTMAX)
    n = 65536
    mb = c.get_microbatch()[1]
    pcm = make_clips(n, 24000, start_index=70000)
    probs = torch.empty((n, 630), dtype=torch.float32, device='cuda')
    am = torch.empty(n, dtype=torch.int32, device='cuda')
    c.si_pipeline_dev(pcm.data_ptr(), n, 24000, 24000, probs.data_ptr(), am.data_ptr())
    c.synchronize()
    idx = _sample(n, min(mb, n), 32, 2) + [n // 2 - 1, n // 2]
    idx = sorted(set(idx))
    sub = pcm[idx].cpu().numpy()
    probs = probs[idx].cpu().numpy()
    am = am[idx].cpu().numpy()
    c.release_workspace()
    p1, a1, _ = c.si_pipeline(sub)        # a small batch: the same per-clip kernels
    assert np.array_equal(p1, probs) and np.array_equal(a1, am)
    rows = list(range(0, len(idx), max(1, len(idx) // 10)))
    x = np.concatenate([si_fe.input_feature_gen(sub[j]) for j in rows]).astype(np.float32)
    ref = nets.si_forward(x, W)
    err = compare.logp_err(probs[rows], ref)
    assert err <= compare.LOGP_TOL, err
    assert compare.argmax_ok(probs[rows], ref) and np.array_equal(am[rows], probs[rows].argmax(1))
    assert compare.near_ties(ref).mean() < 0.05
