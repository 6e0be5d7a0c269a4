"""Offline OD segmentation + batched prediction on the GPU.

predict_segments runs every window of a conversation in one fused call over strided (overlapping)
views of the PCM; each window must give exactly what the per-window pipeline gives (same kernels,
same bytes), and agree with the oracle like test_od_pipeline_matches_features_then_forward.
"""
import numpy as np
import pytest

from oracle import nets, od_fe, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def model():
    from mmla_audio_amd import models, weights
    return models.OverlapDetectionModel(weights.synthetic(weights.OD, seed=11))


@pytest.mark.parametrize('seconds,step', [(6.3, 1.5), (4.0, 0.5), (1.4, 1.5)])
def test_predict_segments_matches_per_window(model, seconds, step):
    from mmla_audio_amd import overlap_detection_post_processing as odpp
    sig = np.concatenate([synth.clip(60 + k, 16000) for k in range(int(np.ceil(seconds)))])
    sig = sig[:int(16000 * seconds)]
    probs, am, labels = odpp.predict_segments(sig, model, 16000, 1.5, step)
    win, st, n = odpp.segment_bounds(sig.size, 16000, 1.5, step)
    assert probs.shape == (n, 2) and len(labels) == n
    if n == 0:
        return
    windows = np.stack([sig[j * st: j * st + win] for j in range(n)])
    p2, am2, _ = model.predict_wavs(windows)
    assert np.array_equal(probs, p2)
    assert np.array_equal(am, am2)
    assert labels == [odpp.OVERLAP_DEGREE[str(k)] for k in am2]
    ref = nets.od_forward(np.stack([od_fe.od_features(w)['png_rgb'] for w in windows[:3]]).astype(
        np.float32), model.W)
    assert np.abs(probs[:3] - ref).max() <= 1e-3


def test_strided_host_path_bounds(model):
    from mmla_audio_amd import _lib
    sig = synth.clip(70, 30000)
    with pytest.raises(_lib.MmlaError):
        model.ctx.od_pipeline_strided(sig, 3, 8000, 24000)     # last window runs past the end
