"""Out-of-bounds stores: every workspace slot framed by guard bands (MMLA_WS_GUARD=1, capi.cpp
ws_get); a call fails if any kernel wrote into one.  Micro-batches and batch sizes that leave
partial tiles at the end of each buffer, OD and SI pipelines, front-ends and the noise gate."""
import os

import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def gctx():
    from mmla_audio_amd import _lib, weights
    os.environ['MMLA_WS_GUARD'] = '1'
    try:
        c = _lib.Context(0)
        c.load_weights(weights.OD, weights.pack(weights.OD, weights.synthetic(weights.OD, seed=31)), 2)
        Ws = weights.synthetic(weights.SI, seed=32, n_classes=8)
        c.load_weights(weights.SI, weights.pack(weights.SI, Ws, 8), 8, 1)
        yield c
    finally:
        os.environ.pop('MMLA_WS_GUARD', None)


@pytest.mark.parametrize('mb,n', [(32, 75), (64, 150), (0, 37)])
def test_od_guards(gctx, mb, n):
    pcm = synth.batch(960 + n, n, 40000)
    gctx.set_microbatch(mb, 0)
    try:
        gctx.od_features(pcm)
        p, a, _ = gctx.od_pipeline(pcm)
    finally:
        gctx.set_microbatch(0, 0)
    assert np.isfinite(p).all()


@pytest.mark.parametrize('mb,n', [(16, 41), (0, 23)])
def test_si_guards(gctx, mb, n):
    pcm = synth.batch(970 + n, n, 24000)
    gctx.set_microbatch(0, mb)
    try:
        gctx.si_features(pcm)
        p, a, s = gctx.si_pipeline(pcm)
    finally:
        gctx.set_microbatch(0, 0)
    assert np.isfinite(p).all()


def test_noise_gate_guards(gctx):
    rng = np.random.default_rng(5)
    gctx.nr_set_noise((0.01 * rng.standard_normal(16000)).astype(np.float32))
    ys = (0.1 * rng.standard_normal((3, 40000))).astype(np.float32)
    out = gctx.nr_reduce(ys)
    assert out.shape == ys.shape and np.isfinite(out).all()
