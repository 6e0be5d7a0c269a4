"""VERDICT r5 missing #1: the reference's own TensorFlow call-site statements (tests/refsites.py, the
text pinned against /root/reference by test_tf_compat_cpu.py) executed unchanged with
``tf = mmla_audio_amd.tf_compat`` on the GPU path:

* OD real time ``record_on_pc.py:88`` (load) + ``:156-160`` (PNG read -> decode -> stack -> predict ->
  argmax) on the PNG ``generate_zcr_image`` wrote (``:139``), and the offline twin
  ``overlap_detection_post_processing.py:154,204-208``.  The probabilities must equal the fused
  ``model.predict_wavs`` on the same WAV bit for bit (the PNG carries exactly the image the fused
  pipeline feeds its network).
* SI ``record_on_pc.py:77`` (the deployed transfer-learning model) + ``:136-137`` on
  ``input_feature_gen``'s output, and ``speaker_identification_post_processing.py:206,272`` on a
  batch of windows: equal to ``predict_wavs`` bit for bit.

The models load trained-layout bundles written by tests/tfbundle_writer.py (seeded weights): the
load statements run verbatim, with no allow_synthetic escape."""
import os

import numpy as np
import pytest
import scipy.io.wavfile as wavfile

import refsites

pytestmark = pytest.mark.gpu


def _wav(path, pcm):
    wavfile.write(path, 16000, np.asarray(pcm, np.int16))
    return path


def test_od_call_sites_verbatim(tmp_path):
    from mmla_audio_amd import tf_compat as tf, weights
    from mmla_audio_amd.overlap_features_generator import OverlapFeaturesGenerator
    from oracle import synth
    from tfbundle_writer import base_keys, write_bundle
    model_path = str(tmp_path / 'timit' / 'models' / 'timit2.0')
    write_bundle(model_path, base_keys(weights.OD, weights.synthetic(weights.OD, seed=11)))
    model = refsites.run(refsites.OD_LOAD, tf=tf, model_path=model_path)['model']
    assert not model.synthetic
    model_off = refsites.run(refsites.OD_OFFLINE_LOAD, tf=tf, model_path=model_path)['model']
    ofg = OverlapFeaturesGenerator(wl=25, hl=10)
    c_png_dir = str(tmp_path / 'png') + '/'
    keys = set()
    for i, n in enumerate((40960, 40000, 24000, 17000, 6000)):   # 2.56 s real time ... short clips
        pcm = synth.clip(7100 + i, n)
        wav = _wav(str(tmp_path / f'{i}.wav'), pcm)
        ofg.generate_zcr_image(wav, c_png_dir, f'{i}.png')                 # record_on_pc.py:139
        ns = refsites.run(refsites.OD_REALTIME, tf=tf, np=np, model=model,
                          features_image_path2=c_png_dir + f'{i}.png')
        probs, am, silent = model.predict_wavs(pcm[None])
        assert ns['_input'].shape == (1, 128, 151, 3) and ns['_input'].dtype == np.float32
        assert ns['prob'].shape == (1, 2) and ns['prob'].dtype == np.float32
        assert np.array_equal(ns['prob'], probs), (i, ns['prob'], probs)
        assert ns['key'] == str(am[0]) and not silent[0]
        keys.add(ns['key'])
        off = refsites.run(refsites.OD_OFFLINE, tf=tf, model=model_off,
                           features_image_path=c_png_dir + f'{i}.png')
        assert np.array_equal(off['prob'], probs)
    assert keys <= {'0', '1'}


def test_si_call_sites_verbatim(tmp_path):
    from mmla_audio_amd import tf_compat as tf, weights
    from mmla_audio_amd import speaker_identification as vi
    from oracle import synth
    from tfbundle_writer import deployed_keys, write_bundle
    k = 5
    model_path = str(tmp_path / 'experiment' / 'model')
    write_bundle(model_path, deployed_keys(weights.synthetic(weights.SI, seed=12, n_classes=k), k,
                                           trainable_first=True))
    model = refsites.run(refsites.SI_LOAD, tf=tf, model_path=model_path)['model']
    assert not model.synthetic and model.n_classes == k
    pcms = [synth.clip(7200 + i, n) for i, n in enumerate((40960, 24000, 41000, 5000))]
    xs = []
    for i, pcm in enumerate(pcms):
        filepath = _wav(str(tmp_path / f'si{i}.wav'), pcm)
        x = vi.input_feature_gen(filepath)                                   # record_on_pc.py:120
        ns = refsites.run(refsites.SI_REALTIME, np=np, model=model, x=x)
        probs, am, silent = model.predict_wavs(pcm[None])
        assert ns['prob'].shape == (1, k)
        assert np.array_equal(ns['prob'], probs), i
        assert ns['key'] == str(am[0])
        xs.append(x[0])
    model_off = refsites.run(refsites.SI_OFFLINE_LOAD, tf=tf, model_path=model_path)['model']
    test_x = np.asarray(xs)
    results = refsites.run(refsites.SI_OFFLINE, model=model_off, test_x=test_x)['results']
    assert results.shape == (len(xs), k)
    for i, pcm in enumerate(pcms):
        assert np.array_equal(results[i], model.predict_wavs(pcm[None])[0][0]), i
