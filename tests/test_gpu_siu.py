"""The fused SI res unit (siu.hip: Conv1D -> BN -> ReLU -> Conv1D + residual in one launch, t1 kept in
LDS) against the two conv_h3 launches it replaces: bit-identical SI probabilities over a batch with
ragged and 'silent' clips, across several tiles and clip boundaries (MMLA_NO_SIU=1 selects the pair)."""
import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu


def _ctx(monkeypatch, fused):
    from mmla_audio_amd import _lib, weights
    monkeypatch.setenv('MMLA_NO_SIU', '0' if fused else '1')
    c = _lib.Context(0)
    monkeypatch.delenv('MMLA_NO_SIU')
    W = weights.synthetic(weights.SI, seed=31, n_classes=630)
    c.load_weights(weights.SI, weights.pack(weights.SI, W, 630), 630, _lib.HEAD_SOFTMAX)
    return c


def test_fused_units_bit_identical(monkeypatch):
    lens = [24000 if i % 9 else (3000 if i % 2 else 17000) for i in range(300)]
    pcm = [synth.clip(4000 + i, n) for i, n in enumerate(lens)]
    p_pair, a_pair, s_pair = _ctx(monkeypatch, False).si_pipeline(pcm)
    p_fused, a_fused, s_fused = _ctx(monkeypatch, True).si_pipeline(pcm)
    assert np.array_equal(p_fused, p_pair) and np.array_equal(a_fused, a_pair)
    assert np.array_equal(s_fused, s_pair)
