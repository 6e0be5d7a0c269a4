"""The drop-in boundary by its reference names, against the golden fixtures that
tests/golden/make_golden.py produced by running the reference's own functions on the same WAVs.

  OverlapFeaturesGenerator(25, 10).generate_mels / generate_zcr / generate_zcr_image
      (overlap_features_generator.py:65-151) incl. the PNG a caller re-reads (record_on_pc.py:156)
  input_feature_gen (speaker_identification.py:372-398): 'silent' sentinel, float64 [1,256,39]
  delta (:141-151), make_feature_experiment (:317-369) with the binarizer's cross-call state
  models.load_model: raises without trained variables unless allow_synthetic=True

Tolerances as tests/test_gpu_parity.py; the PNG: R exact, G/B within 1 LSB on at
most 1e-4 of the pixel values.
"""
import os

import numpy as np
import pytest
import scipy.io.wavfile as wavfile

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, 'tests', 'golden')


def _wav(tmp_path, name, pcm):
    p = str(tmp_path / f'{name}.wav')
    wavfile.write(p, 16000, np.asarray(pcm, np.int16))
    return p


def _png_rgb(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert('RGB'), dtype=np.uint8)


def test_overlap_features_generator_by_reference_names(tmp_path, od_golden):
    from mmla_audio_amd.overlap_features_generator import OverlapFeaturesGenerator
    ofg = OverlapFeaturesGenerator(wl=25, hl=10)
    assert ofg.get_attributes() == (400, 160, 16000)
    out_dir = str(tmp_path / 'png') + '/'
    lsb_px = 0
    for i, name in enumerate(od_golden['names']):
        wav = _wav(tmp_path, f'od{i}', od_golden[f'pcm_{i}'])
        s_db, norm = ofg.generate_mels(wav)
        ref_norm, ref_db = od_golden[f'norm_{i}'], od_golden[f'db_{i}']
        assert s_db.dtype == np.float32 and norm.dtype == np.float32 and norm.shape == (128, 151)
        nan = np.isnan(ref_norm)
        assert np.array_equal(np.isnan(norm), nan), name
        if (~nan).any():
            assert np.abs(norm[~nan] - ref_norm[~nan]).max() <= 1e-4, name
            assert np.abs(s_db - ref_db).max() <= 5e-3, name
        zcr = ofg.generate_zcr(wav)
        assert zcr.dtype == np.float64 and zcr.shape == (1, 151)
        assert np.array_equal(zcr, od_golden[f'zcr_{i}']), name            # exact counts / 400
        img = ofg.generate_zcr_image(wav, out_dir, None)
        assert img.dtype == np.float64 and img.shape == (128, 151, 3)
        assert np.array_equal(img[..., 0], np.broadcast_to(zcr, (128, 151))), name
        if 'image_0' in od_golden and i == 0:
            assert np.abs(img - od_golden['image_0']).max() <= 1e-4
        assert ofg.generate_zcr_image(wav, out_dir, f'od{i}.png') is None
        got = _png_rgb(out_dir + f'od{i}.png').astype(int)
        want = od_golden[f'png_{i}'].astype(int)
        assert np.array_equal(got[..., 0], want[..., 0]), f'{name}: R channel'
        d = np.abs(got - want)
        assert d.max() <= 1, name
        lsb_px += int(np.count_nonzero(d))
    total = len(od_golden['names']) * 128 * 151 * 3
    assert lsb_px <= 1e-4 * total, f'{lsb_px} of {total} pixel values 1 LSB off'


def test_png_bytes_match_matplotlib(tmp_path, od_golden):
    """generate_zcr_image writes the file plt.imsave(origin='lower') writes for the same pixels"""
    plt = pytest.importorskip('matplotlib.pyplot')
    from mmla_audio_amd.overlap_features_generator import OverlapFeaturesGenerator
    ofg = OverlapFeaturesGenerator(wl=25, hl=10)
    wav = _wav(tmp_path, 'od0', od_golden['pcm_0'])
    ofg.generate_zcr_image(wav, str(tmp_path) + '/', 'ours.png')
    img = ofg.generate_zcr_image(wav, str(tmp_path) + '/', None)
    plt.imsave(str(tmp_path / 'ref.png'), img, origin='lower')   # the reference's call, :151
    ours, ref = open(tmp_path / 'ours.png', 'rb').read(), open(tmp_path / 'ref.png', 'rb').read()
    if _png_rgb(tmp_path / 'ours.png').tobytes() == _png_rgb(tmp_path / 'ref.png').tobytes():
        assert ours == ref


def test_input_feature_gen_by_reference_name(tmp_path, si_golden):
    from mmla_audio_amd.speaker_identification import input_feature_gen
    for i, name in enumerate(si_golden['names']):
        wav = _wav(tmp_path, f'si{i}', si_golden[f'pcm_{i}'])
        x = input_feature_gen(wav)
        if bool(si_golden[f'silent_{i}']):
            assert isinstance(x, str) and x == 'silent', name
            continue
        assert isinstance(x, np.ndarray) and x.dtype == np.float64 and x.shape == (1, 256, 39), name
        assert np.abs(x - si_golden[f'feat_{i}']).max() <= 1e-4, name


def test_delta_shim(si_golden):
    from mmla_audio_amd.speaker_identification import delta
    d = delta(si_golden['delta_in'], 2)
    assert np.allclose(d, si_golden['delta_out'], rtol=0, atol=1e-12)
    assert np.allclose(delta(d, 2), si_golden['delta2_out'], rtol=0, atol=1e-12)


def test_make_feature_experiment_two_calls(tmp_path):
    """chunking, one-hot labels and speaker_id of consecutive calls in one process, including the
    reference binarizer's label collision on the second call"""
    from oracle import synth
    from mmla_audio_amd import speaker_identification as si
    g = np.load(os.path.join(GOLDEN, 'si_experiment_golden.npz'))
    si._speakers_count_dict.clear()   # a fresh process, like the golden run
    k = 0
    while f'x_{k}' in g:
        files = []
        for j, (label, seed, n) in enumerate(zip(g[f'labels_{k}'], g[f'seeds_{k}'], g[f'lens_{k}'])):
            d = tmp_path / f'exp{k}' / str(j)
            d.mkdir(parents=True)
            files.append(_wav(d, str(label), synth.clip(int(seed), int(n))))
        x, y, spk = si.make_feature_experiment(files)
        assert x.dtype == np.float64 and x.shape == g[f'x_{k}'].shape
        assert np.abs(x - g[f'x_{k}']).max() <= 1e-4
        assert np.array_equal(y, g[f'y_{k}'])
        assert sorted(spk.items()) == [tuple(r) for r in g[f'speaker_id_{k}'].tolist()]
        k += 1
    assert k == 2


def test_load_model_requires_trained_weights(tmp_path):
    from mmla_audio_amd import models
    d = tmp_path / 'timit2.0'
    (d / 'variables').mkdir(parents=True)
    idx = os.path.join(GOLDEN, 'od_timit2.0_variables.index')
    (d / 'variables' / 'variables.index').write_bytes(open(idx, 'rb').read())
    with pytest.raises(FileNotFoundError):
        models.load_model(str(d))
    with pytest.warns(UserWarning):
        m = models.load_model(str(d), allow_synthetic=True)
    assert m.synthetic and m.predict(np.zeros((1, 128, 151, 3), np.float32)).shape == (1, 2)
