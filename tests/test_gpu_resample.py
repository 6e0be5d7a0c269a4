"""GPU rate conversion (resample.hip) through the C ABI.

mmla_ratecv against stdlib audioop.ratecv (what pydub's set_frame_rate calls,
overlap_detection_post_processing.py:120-121, speaker_identification_post_processing.py:159-160):
bit-identical.  mmla_resample_sinc against the oracle's resampy restatement with the same filter
table: bit-identical (resampy itself is absent: parity with the library unpinned).
"""
import math
import warnings

import numpy as np
import pytest

from oracle import resample as ors

with warnings.catch_warnings():
    warnings.simplefilter('ignore', DeprecationWarning)
    import audioop

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from mmla_audio_amd import _lib
    return _lib.Context(0)


@pytest.mark.parametrize('ir,orr', [(48000, 16000), (44100, 16000), (22050, 16000), (32000, 16000),
                                    (8000, 16000), (16000, 22050), (11025, 16000)])
@pytest.mark.parametrize('nch', [1, 2])
def test_ratecv_matches_audioop(ctx, ir, orr, nch):
    rng = np.random.default_rng(ir + 7 * orr + nch)
    for n in (1, 2, 3, 1000, 48000 * 3 + 7):
        x = (rng.standard_normal(n * nch) * 9000).clip(-32768, 32767).astype('<i2')
        x[:4] = [32767, -32768, -1, 1][:min(4, x.size)]
        want = np.frombuffer(audioop.ratecv(x.tobytes(), 2, nch, ir, orr, None)[0], '<i2')
        got = ctx.ratecv(x, nch, ir, orr)
        assert np.array_equal(got, want), (ir, orr, nch, n)
    assert ctx.ratecv(np.zeros(0, np.int16), nch, ir, orr).size == 0


def test_audio_segment_set_frame_rate(ctx):
    from mmla_audio_amd.audio_segment import AudioSegment
    rng = np.random.default_rng(5)
    x = (rng.standard_normal(2 * 48000) * 5000).astype('<i2')      # 1 s of 48 kHz stereo
    seg = AudioSegment(x, 48000, 2, ctx).set_frame_rate(16000)
    want = np.frombuffer(audioop.ratecv(x.tobytes(), 2, 2, 48000, 16000, None)[0], '<i2')
    assert seg.frame_rate == 16000 and seg.channels == 2 and np.array_equal(seg.data, want)


@pytest.mark.parametrize('sr0,sr1', [(16000, 22050), (22050, 16000), (48000, 22050), (8000, 22050)])
def test_resample_sinc_matches_restatement(ctx, sr0, sr1):
    from mmla_audio_amd.audio_segment import kaiser_best_table, resample
    table = kaiser_best_table()
    rng = np.random.default_rng(sr0 + sr1)
    for n in (1, 5, 700, 2 * sr0 + 13):
        x = (rng.standard_normal(n) * 0.2).astype(np.float32)
        got = ctx.resample_sinc(x, sr0, sr1, *table)
        want = ors.resample_kaiser_best(x, sr0, sr1, table)
        assert got.shape == want.shape
        assert np.array_equal(got, want), (sr0, sr1, n, np.abs(got - want).max())
    y = resample(x, sr0, sr1, ctx)                      # + librosa's fix_length
    assert np.array_equal(y, ors.librosa_resample(x, sr0, sr1, table))


@pytest.mark.parametrize('dbfs', [-20, -3.5])
def test_od_standardize_audio_gain(ctx, tmp_path, dbfs):
    """OD standardize_audio(source, target, format, dbfs) with a gain target (the reference's
    post_anlysing passes dbfs=0, which skips it): pydub set_frame_rate -> apply_gain(dbfs - dBFS)
    -> export, i.e. audioop.ratecv -> audioop.rms -> audioop.mul, byte for byte
    (overlap_detection_post_processing.py:101-125)"""
    import wave
    from mmla_audio_amd.overlap_detection_post_processing import standardize_audio
    rng = np.random.default_rng(11)
    x = (rng.standard_normal(2 * 44100) * 3000).clip(-32768, 32767).astype('<i2')   # 1 s stereo
    src, dst = str(tmp_path / 'zoom_a.wav'), str(tmp_path / 'zoom_a_std.wav')
    with wave.open(src, 'wb') as f:
        f.setnchannels(2)
        f.setsampwidth(2)
        f.setframerate(44100)
        f.writeframes(x.tobytes())
    pcm = standardize_audio(src, dst, None, dbfs, ctx=ctx)
    conv = audioop.ratecv(x.tobytes(), 2, 2, 44100, 16000, None)[0]
    level = 20 * math.log(audioop.rms(conv, 2) / 32768.0, 10)   # pydub ratio_to_db
    want = np.frombuffer(audioop.mul(conv, 2, 10 ** ((dbfs - level) / 20)), '<i2')
    assert np.array_equal(pcm, want)
    with wave.open(dst, 'rb') as f:
        assert (f.getnchannels(), f.getframerate()) == (2, 16000)
        assert np.array_equal(np.frombuffer(f.readframes(f.getnframes()), '<i2'), want)
