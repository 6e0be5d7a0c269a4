"""OD res_blocks 4-9 as one fused kernel each (odu.hip: t1 kept in LDS, full-height column strips)
against the conv_h3 pairs they replace (env MMLA_NO_ODU=1): bit for bit at every block output
(debug trace), through the whole pipeline, with ragged clip counts and the range guard tripped.
Reference: OverlapDetection/scripts/overlap_detector_temp.py:253-277 (res_block)."""
import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu


def _ctx(monkeypatch, odu, W):
    from mmla_audio_amd import _lib, weights
    monkeypatch.setenv('MMLA_NO_ODU', '0' if odu else '1')
    c = _lib.Context(0)
    monkeypatch.delenv('MMLA_NO_ODU')
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    return c


@pytest.mark.parametrize('seed', [41, 42])
def test_odu_bit_identical_blocks(monkeypatch, seed):
    from mmla_audio_amd import weights
    W = weights.synthetic(weights.OD, seed=seed)
    fused, pair = _ctx(monkeypatch, True, W), _ctx(monkeypatch, False, W)
    pcm = synth.batch(3000 + seed, 5, 40000)
    img = fused.od_features(pcm, db=False, norm=False, zcr=False)['img'].astype(np.float32)
    assert np.array_equal(img, pair.od_features(pcm, db=False, norm=False, zcr=False)['img'])
    for stage in range(4, 12):
        a, b = fused.debug_od_trace(img, stage), pair.debug_od_trace(img, stage)
        assert np.isfinite(a).all(), stage
        assert np.array_equal(a, b), (stage, float(np.abs(a - b).max()))


@pytest.mark.parametrize('n', [1, 7, 133])
def test_odu_pipeline_bit_identical(monkeypatch, n):
    from mmla_audio_amd import weights
    W = weights.synthetic(weights.OD, seed=43)
    fused, pair = _ctx(monkeypatch, True, W), _ctx(monkeypatch, False, W)
    pcm = synth.batch(3100 + n, n, 40000)
    pf, af, _ = fused.od_pipeline(pcm)
    pp, ap, _ = pair.od_pipeline(pcm)
    assert np.array_equal(pf, pp) and np.array_equal(af, ap)
    assert fused.range_check() == 0 and pair.range_check() == 0


def test_odu_range_guard(monkeypatch):
    """block 4's input scaled past the fp16 split range: the fused kernel flags it like the pair, and
    the host call re-runs in exact f32 (same result both ways)"""
    from mmla_audio_amd import weights
    W = weights.synthetic(weights.OD, seed=44)
    for k in ('layer_with_weights-14/moving_variance',):   # BN_in of block 4 (lww 14..18)
        assert k in W
    W = dict(W)
    # BN_mid of block 3's conv(4,1) input unchanged; scale block 4's BN_in output instead: gamma x 1e4
    W['layer_with_weights-14/gamma'] = W['layer_with_weights-14/gamma'] * 1e4
    fused, pair = _ctx(monkeypatch, True, W), _ctx(monkeypatch, False, W)
    pcm = synth.batch(3200, 3, 40000)
    pf, _, _ = fused.od_pipeline(pcm)
    pp, _, _ = pair.od_pipeline(pcm)
    assert fused.range_check() >= 1 and pair.range_check() >= 1
    assert np.array_equal(pf, pp)
