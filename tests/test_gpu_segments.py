"""Offline OD segmentation + batched prediction on the GPU.

predict_segments runs every window of a conversation in one fused call over strided (overlapping)
views of the PCM; each window must give exactly what the per-window pipeline gives (same kernels,
same bytes), and agree with the oracle like test_od_pipeline_matches_features_then_forward.
"""
import numpy as np
import pytest

from oracle import compare, nets, od_fe, synth

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
    # the log-probability bar (oracle/compare.py): 1e-4 against the float64 OD-NET on the GPU's own
    # images, 1e-3 end to end against the oracle front-end (images may differ by 1 LSB on a few pixels)
    f = model.ctx.od_features(windows[:3], db=False, norm=False, zcr=False)
    assert compare.logp_err(probs[:3], nets.od_forward(f['img'].astype(np.float32), model.W)) <= compare.LOGP_TOL
    ref = nets.od_forward(np.stack([od_fe.od_features(w)['png_rgb'] for w in windows[:3]]).astype(
        np.float32), model.W)
    assert compare.logp_err(probs[:3], ref) <= 1e-3
    assert compare.argmax_ok(probs[:3], ref)


def test_strided_host_path_bounds(model):
    from mmla_audio_amd import _lib
    sig = synth.clip(70, 30000)
    with pytest.raises(_lib.MmlaError):
        model.ctx.od_pipeline_strided(sig, 3, 8000, 24000)     # last window runs past the end


def test_post_anlysing_chain_matches_reference(tmp_path):
    """the OD offline chain (overlap_detection_post_processing.py:151-226) --
    standardise (3 stationary noise-gate passes + PCM_16 rewrites for audio*, none for zoom*),
    1.5 s segmentation, one fused features + OD-NET call per conversation, TSV log -- against the
    reference's own post_anlysing run with stubs (tests/golden/odpost_golden.npz, make_golden.py
    'odpost'; the float64 oracle OD-NET with the seed-0 synthetic weights stands in for Keras).
    The standardised PCM agrees to the noise gate's rounding ties; the log lists segments in this directory's os.listdir order, so it is rebuilt from the reference's
    per-segment labels in that order."""
    import datetime
    import os
    import scipy.io.wavfile as wavfile
    from mmla_audio_amd import models, weights, overlap_detection_post_processing as odpp
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'odpost_golden.npz'))
    root = str(tmp_path)
    pt = os.path.join(root, 'experiment', 'recordings', 'post-time')
    for d in ('whole', 'standardized', 'segments', 'features'):
        os.makedirs(os.path.join(pt, d))
    os.makedirs(os.path.join(root, 'experiment', 'logs'))
    wavfile.write(os.path.join(root, 'experiment', 'Ambient_Noise.wav'), 16000, g['noise'])
    names = list(g['names'])
    for i, name in enumerate(names):      # zoom_conv2: a 48 kHz stereo export
        wavfile.write(os.path.join(pt, 'whole', name), int(g[f'rate_{i}']), g[f'pcm_{i}'])
    model = models.OverlapDetectionModel(weights.synthetic(weights.OD, seed=0))
    t0 = datetime.datetime(2026, 10, 17, 9, 30, 0)
    out = odpp.post_anlysing(root, model, start_time=t0)
    from PIL import Image
    for i, name in enumerate(names):
        stem = name[:-4]
        rate, std = wavfile.read(os.path.join(pt, 'standardized', name))
        assert rate == 16000 and std.shape == g[f'std_{i}'].shape, name
        if name.startswith('zoom'):
            # pydub set_frame_rate = audioop.ratecv (mmla_ratecv), stereo kept: the same samples
            assert np.array_equal(std, g[f'std_{i}']), name
        else:
            # nr.hip equals the restated gate to ~1e-7 of the peak on 99.9 % of the samples, with
            # rare mask-threshold flips (test_gpu_vad.py::test_save_wave_file_chain: 1e-5 / 2e-2)
            d = np.abs(std.astype(np.int64) - g[f'std_{i}'].astype(np.int64))
            assert np.mean(d > 0) <= 1e-3, name
            assert np.quantile(d, 0.999) <= 1 and d.max() <= 0.02 * 32767, name
        # the features/<conversation>/<count>.png images of generate_zcr_image (:201-203)
        fdir = os.path.join(pt, 'features', stem)
        assert len(os.listdir(fdir)) == int(g[f'png_count_{i}']), name
        k = os.listdir(os.path.join(pt, 'segments', stem)).index(str(g[f'listing_{i}'][0]))
        got = np.asarray(Image.open(os.path.join(fdir, f'{k}.png')).convert('RGB'), np.int16)
        want = np.asarray(Image.open(__import__('io').BytesIO(g[f'png0_{i}'].tobytes())).convert('RGB'), np.int16)
        assert got.shape == want.shape and np.abs(got - want).max() <= 1, name
        want = dict(zip(g[f'seg_names_{i}'], g[f'seg_labels_{i}']))
        listing = os.listdir(os.path.join(pt, 'segments', stem))
        assert sorted(listing) == sorted(want)
        assert dict(out[name]) == want, name
        lines = ['segment\toverlapped degree\ttimestamp']
        for count, f in enumerate(listing):
            lines.append(f'{count}\t{want[f]}\t{t0 + datetime.timedelta(seconds=1.5 * count)}')
        log = open(os.path.join(root, 'experiment', 'logs', stem + '.txt')).read()
        assert log == '\n'.join(lines) + '\n'
        if list(listing) == list(g[f'listing_{i}']):       # same directory order: the very bytes
            assert log == str(g[f'log_{i}'])


def test_offline_labels_map_silent_windows(model):
    """a window shorter than 4000 samples comes back as argmax -1; the labels and the
    log map it to 'silent' (record_on_pc.py:141-154) instead of raising KeyError."""
    from mmla_audio_amd import overlap_detection_post_processing as odpp
    sig = synth.clip(71, 3000)
    model._ensure_loaded()
    probs, am = model.ctx.od_pipeline_strided(sig, 1, 3000, 3000)
    assert int(am[0]) == -1
    assert odpp.LABELS[str(int(am[0]))] == 'silent'
