"""The fused SI res units (siu.hip) against the conv_h3 launches they replace: bit-identical SI
probabilities over a batch with ragged and 'silent' clips, across several tiles and clip boundaries.

* MMLA_NO_SIU: units without pooling (Conv1D -> BN -> ReLU -> Conv1D + residual, t1 kept in LDS);
* MMLA_NO_SIPU: the pool units (MaxPool1D in the staging, the stride-2 shortcut in the epilogue);
* MMLA_NO_SIFIN: the last unit writing the final BN + ReLU + AveragePooling1D(4) itself;
* MMLA_NO_SIPAD: si_fe's 40-float feature rows (zero 40th column) read by the stem as float4;
* MMLA_NO_SIPAIR: two consecutive units without pooling as one kernel (the first unit's output kept
  on chip), with and without the last unit's fused pooling;
* MMLA_NO_SICHAIN: a pool unit and the two units after it as one kernel.
Each switch is set explicitly, so the tests hold whatever the library's defaults are."""
import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu

ALL_ON = {'MMLA_NO_SIU': '0', 'MMLA_NO_SIPU': '0', 'MMLA_NO_SIFIN': '0', 'MMLA_NO_SIPAD': '0',
          'MMLA_NO_SIPAIR': '0', 'MMLA_NO_SICHAIN': '0'}
ALL_OFF = {'MMLA_NO_SIU': '1', 'MMLA_NO_SIPU': '1', 'MMLA_NO_SIFIN': '1', 'MMLA_NO_SIPAD': '1',
           'MMLA_NO_SIPAIR': '1', 'MMLA_NO_SICHAIN': '1'}


def _ctx(monkeypatch, env):
    from mmla_audio_amd import _lib, weights
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    c = _lib.Context(0)
    for k in env:
        monkeypatch.delenv(k)
    W = weights.synthetic(weights.SI, seed=31, n_classes=630)
    c.load_weights(weights.SI, weights.pack(weights.SI, W, 630), 630, _lib.HEAD_SOFTMAX)
    return c


@pytest.fixture(scope='module')
def pcm():
    lens = [24000 if i % 9 else (3000 if i % 2 else 17000) for i in range(300)]
    return [synth.clip(4000 + i, n) for i, n in enumerate(lens)]


def _same(monkeypatch, pcm, env_a, env_b):
    p_a, a_a, s_a = _ctx(monkeypatch, env_a).si_pipeline(pcm)
    p_b, a_b, s_b = _ctx(monkeypatch, env_b).si_pipeline(pcm)
    assert np.array_equal(p_a, p_b) and np.array_equal(a_a, a_b)
    assert np.array_equal(s_a, s_b)


def test_fused_units_bit_identical(monkeypatch, pcm):
    _same(monkeypatch, pcm, ALL_ON, ALL_OFF)


def test_fused_pool_units_bit_identical(monkeypatch, pcm):
    _same(monkeypatch, pcm, ALL_ON, dict(ALL_ON, MMLA_NO_SIPU='1'))


def test_fused_final_pool_bit_identical(monkeypatch, pcm):
    _same(monkeypatch, pcm, ALL_ON, dict(ALL_ON, MMLA_NO_SIFIN='1'))


def test_padded_feature_rows_bit_identical(monkeypatch, pcm):
    _same(monkeypatch, pcm, ALL_ON, dict(ALL_ON, MMLA_NO_SIPAD='1'))


def test_unit_pairs_bit_identical(monkeypatch, pcm):
    no_chain = dict(ALL_ON, MMLA_NO_SICHAIN='1')
    _same(monkeypatch, pcm, no_chain, dict(no_chain, MMLA_NO_SIPAIR='1'))
    _same(monkeypatch, pcm, dict(no_chain, MMLA_NO_SIFIN='1'), dict(no_chain, MMLA_NO_SIPAIR='1', MMLA_NO_SIFIN='1'))


def test_unit_chains_bit_identical(monkeypatch, pcm):
    _same(monkeypatch, pcm, ALL_ON, dict(ALL_ON, MMLA_NO_SICHAIN='1'))
    _same(monkeypatch, pcm, dict(ALL_ON, MMLA_NO_SIFIN='1'), dict(ALL_ON, MMLA_NO_SICHAIN='1', MMLA_NO_SIFIN='1'))


@pytest.mark.parametrize('n', [1, 2, 5])
def test_unit_pairs_small_batches(monkeypatch, pcm, n):
    """batches smaller than one pair workgroup's rows (every row clamped at both batch ends)"""
    _same(monkeypatch, pcm[:n], ALL_ON, ALL_OFF)
