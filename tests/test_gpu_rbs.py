"""OD res_blocks 1-3 as rolling column strips (rbs.hip, 32x32x16 MFMAs) against the 16 x 16 tile
kernels they replace (resblk.hip, env MMLA_RB_TILE=1) and the float64 oracle: the block outputs
(debug trace stages 1-3) agree to float32 rounding -- the two kernels sum the same 3xFP16 products
in a different MFMA order, so not bit for bit --, the pipeline's probabilities and labels agree, the
u8 and float image entries give the same bits, ragged clip counts cross strip / chunk edges, and the
range guard trips in the strips like in the tiles.
Reference: OverlapDetection/scripts/overlap_detector_temp.py:253-303 (stem + res_blocks 1-3)."""
import numpy as np
import pytest

from oracle import nets, synth

pytestmark = pytest.mark.gpu


def _ctx(monkeypatch, strips, W):
    from mmla_audio_amd import _lib, weights
    monkeypatch.setenv('MMLA_RB_TILE', '0' if strips else '1')
    c = _lib.Context(0)
    monkeypatch.delenv('MMLA_RB_TILE')
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    return c


def _oracle_blocks(x, W, upto=3):
    x = np.asarray(x, np.float64)
    net = nets._conv(x, W, 0)
    out, k = {}, 1
    for b in range(upto):
        pool = nets.POOL[b]
        o = nets._conv(nets.elu(nets.batchnorm(net, W, k)), W, k + 1)
        o = nets._conv(nets.elu(nets.batchnorm(o, W, k + 2)), W, k + 3)
        if pool:
            res = nets._conv(net, W, k + 4, stride=2)
            o = nets.maxpool2d_same(o)
            k += 5
        else:
            res = net
            k += 4
        net = res + o
        out[b + 1] = net
    return out


@pytest.mark.parametrize('seed', [51, 52])
def test_rbs_blocks_match_tiles_and_oracle(monkeypatch, seed):
    from mmla_audio_amd import weights
    W = weights.synthetic(weights.OD, seed=seed)
    strips, tiles = _ctx(monkeypatch, True, W), _ctx(monkeypatch, False, W)
    x = np.random.default_rng(seed).integers(0, 256, size=(3, 128, 151, 3)).astype(np.float32)
    ref = _oracle_blocks(x, W)
    for stage in (1, 2, 3):
        a, b = strips.debug_od_trace(x, stage), tiles.debug_od_trace(x, stage)
        assert np.isfinite(a).all(), stage
        scale = float(np.abs(ref[stage]).max())
        assert float(np.abs(a - b).max()) <= 2e-6 * scale, (stage, float(np.abs(a - b).max()) / scale)
        assert float(np.abs(a - ref[stage]).max()) <= 1e-5 * scale, stage


@pytest.mark.parametrize('n', [1, 7, 133])
def test_rbs_pipeline_matches_tiles(monkeypatch, n):
    from mmla_audio_amd import weights
    from oracle import compare
    W = weights.synthetic(weights.OD, seed=53)
    strips, tiles = _ctx(monkeypatch, True, W), _ctx(monkeypatch, False, W)
    pcm = synth.batch(3300 + n, n, 40000)
    ps, a_s, _ = strips.od_pipeline(pcm)
    pt, a_t, _ = tiles.od_pipeline(pcm)
    assert compare.logp_err(ps, pt.astype(np.float64)) <= 1e-5
    agree, disagree, _ = compare.argmax_report(ps, pt.astype(np.float64))
    assert disagree == 0
    assert strips.range_check() == 0


def test_rbs_u8_and_float_images_identical(monkeypatch):
    from mmla_audio_amd import weights
    W = weights.synthetic(weights.OD, seed=54)
    c = _ctx(monkeypatch, True, W)
    img = np.random.default_rng(54).integers(0, 256, size=(5, 128, 151, 3)).astype(np.uint8)
    pf = c.od_forward(img.astype(np.float32))
    pu = c.od_forward(img)
    assert np.array_equal(pf, pu)


def test_rbs_range_guard(monkeypatch):
    """block 2's BN_in scaled past the split range: the strips flag it, the host call re-runs the
    micro-batch in exact f32 -- the same bits as the tile kernels' re-run"""
    from mmla_audio_amd import weights
    W = dict(weights.synthetic(weights.OD, seed=55))
    W['layer_with_weights-6/gamma'] = W['layer_with_weights-6/gamma'] * 1e5   # block 2 BN_in
    strips, tiles = _ctx(monkeypatch, True, W), _ctx(monkeypatch, False, W)
    pcm = synth.batch(3400, 3, 40000)
    ps, _, _ = strips.od_pipeline(pcm)
    pt, _, _ = tiles.od_pipeline(pcm)
    assert strips.range_check() >= 1 and tiles.range_check() >= 1
    assert np.array_equal(ps, pt)
