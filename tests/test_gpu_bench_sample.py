"""The bench's headline parity sample, pinned.

bench.py's `od_pipeline` line compares the GPU pipeline with the float64 oracle on 32 clips of its
65 536-clip batch (first / last clip of every 16 384-clip micro-batch + 24 seeded random clips),
seed-0 synthetic weights.  Its end-to-end log-probability error carries two sources: the network's
arithmetic and the image's permitted 1-LSB pixel values (<= 1 LSB on <= 1e-4 of the
pixel values), which the seeded network amplifies -- in round 4 four such pixel values of clip
52 307 moved its log-probability by 1.6e-4 while the network on the GPU's own image stayed within
3e-7 (tools/parity_drift.py / parity_drift_report.py).  This test pins the two separately on the
same clips: the network on the GPU image against the oracle network on that image (<= 1e-4, in
both arithmetics), and the GPU image against the oracle image (R exact, G/B <= 1 LSB, within the
pixel budget).  Reference: OverlapDetection/scripts/overlap_detector_temp.py:253-303 (the graph),
overlap_features_generator.py:133-151 (the image), tfl_convert.py:73-87 (argmax parity).
"""
import numpy as np
import pytest

from oracle import compare, od_fe
from oracle.nets_torch import Nets

pytestmark = pytest.mark.gpu

N, MB, K_RANDOM, SEED = 65536, 16384, 24, 20261015


def bench_sample_indices():
    """bench.sample_indices(65536, 16384, 24)"""
    idx = set()
    for c0 in range(0, N, MB):
        idx.update((c0, min(c0 + MB, N) - 1))
    idx.update(np.random.default_rng(SEED).choice(N, K_RANDOM, replace=False).tolist())
    return sorted(idx)


@pytest.fixture(scope='module')
def sample():
    import torch
    from mmla_audio_amd.synthetic import make_clips
    idx = bench_sample_indices()
    pcm = make_clips(N, 40000)           # the bench's batch (rank 0), generated in HBM
    sub = pcm[idx].contiguous()
    del pcm
    torch.cuda.empty_cache()
    return idx, sub


def test_bench_sample_net_and_image(sample):
    import torch
    from mmla_audio_amd import _lib, weights
    idx, sub = sample
    n = len(idx)
    c = _lib.Context(0)
    W = weights.synthetic(weights.OD, seed=0)
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    c.set_stream(torch.cuda.current_stream().cuda_stream)
    img = torch.empty((n, 128, 151, 3), dtype=torch.uint8, device='cuda')
    probs = torch.empty((n, 2), dtype=torch.float32, device='cuda')
    c.od_features_dev(sub.data_ptr(), n, 40000, 40000, img=img.data_ptr())
    c.od_pipeline_dev(sub.data_ptr(), n, 40000, 40000, probs=probs.data_ptr())
    c.synchronize()
    gimg = img.cpu().numpy()
    gp = probs.cpu().numpy()
    host = sub.cpu().numpy()
    # the fused pipeline's network reads exactly this image
    assert np.array_equal(gp, c.od_forward(gimg))
    net = Nets(W)
    ref_net = net.od_forward(gimg.astype(np.float32))
    err = compare.logp_err(gp, ref_net)
    assert err <= compare.LOGP_TOL, f'3xFP16 net on the GPU image: log-prob error {err}'
    assert compare.argmax_ok(gp, ref_net)
    c.set_precision(_lib.PREC_F32)
    p32 = c.od_forward(gimg)
    c.set_precision(_lib.PREC_F16X3)
    err32 = compare.logp_err(p32, ref_net)
    assert err32 <= compare.LOGP_TOL, f'f32 net on the GPU image: log-prob error {err32}'
    counts = []
    f = {'img': gimg}
    for j in range(n):
        ref = od_fe.od_features(host[j])
        counts.append(compare.od_clip_compare(f, j, ref, f'bench clip {idx[j]}'))
    compare.od_lsb_budget(counts)
