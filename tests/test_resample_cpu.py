"""CPU: the offline pre-conditioning's rate / level arithmetic pinned against stdlib audioop.

pydub's set_frame_rate, dBFS and apply_gain are audioop.ratecv / audioop.rms / audioop.mul
(OverlapDetection/scripts/overlap_detection_post_processing.py:120-124,
SpeakerIdentification/scripts/speaker_identification_post_processing.py:159-164).  audioop is part of
this image's Python 3.10, so the oracle's closed-form ratecv (which the GPU kernel implements) and the
drop-in's host mul / rms are checked against the real thing here.
"""
import math
import warnings

import numpy as np
import pytest

from oracle import resample as ors

with warnings.catch_warnings():
    warnings.simplefilter('ignore', DeprecationWarning)
    import audioop

RATES = [(48000, 16000), (44100, 16000), (22050, 16000), (32000, 16000), (8000, 16000),
         (16000, 22050), (11025, 16000), (24000, 16000), (16000, 16000)]


def _pcm(rng, n):
    x = (rng.standard_normal(n) * 9000).clip(-32768, 32767).astype('<i2')
    x[:6] = [32767, -32768, 32767, -32768, -1, 1][:min(6, n)]
    return x


@pytest.mark.parametrize('ir,orr', RATES)
@pytest.mark.parametrize('nch', [1, 2])
def test_ratecv_restatement_matches_audioop(ir, orr, nch):
    rng = np.random.default_rng(ir + orr + nch)
    for n in (0, 1, 2, 3, 5, 480, 4801):
        x = _pcm(rng, n * nch)
        want = np.frombuffer(audioop.ratecv(x.tobytes(), 2, nch, ir, orr, None)[0], '<i2')
        got = ors.ratecv(x, nch, ir, orr)
        assert len(want) == ors.ratecv_len(n, ir, orr) * nch
        assert np.array_equal(got, want), (ir, orr, nch, n)


def test_mul_and_rms_match_audioop():
    from mmla_audio_amd.audio_segment import AudioSegment, mul
    rng = np.random.default_rng(3)
    x = _pcm(rng, 20001)
    for factor in (0.0, 0.1, 0.5, 1.0, 10 ** (-20 / 20), 10 ** (7.3 / 20), 3.9, 1e3):
        want = np.frombuffer(audioop.mul(x.tobytes(), 2, factor), '<i2')
        assert np.array_equal(mul(x, factor), want), factor
    for pcm in (x, np.zeros(100, np.int16), np.array([1, -1, 2], np.int16)):
        seg = AudioSegment(pcm, 16000)
        assert seg.rms == audioop.rms(pcm.astype('<i2').tobytes(), 2)
    seg = AudioSegment(x, 16000)
    # pydub: dBFS = 20 math.log(rms / 2^15, 10); apply_gain(d) = mul by 10^(d/20)
    assert seg.dBFS == 20 * math.log(audioop.rms(x.tobytes(), 2) / 32768.0, 10)   # pydub ratio_to_db
    g = seg.apply_gain(-20 - seg.dBFS)
    want = np.frombuffer(audioop.mul(x.tobytes(), 2, 10 ** ((-20 - seg.dBFS) / 20)), '<i2')
    assert np.array_equal(g.data, want)
    assert AudioSegment(np.zeros(10, np.int16), 16000).dBFS == -float('inf')


def test_kaiser_best_table_numpy_vs_scipy():
    """resampy built kaiser_best with scipy's Kaiser window; numpy's agrees to the last bits"""
    a, na = ors.kaiser_best_table('numpy')
    b, nb = ors.kaiser_best_table('scipy')
    assert na == nb == 512 and len(a) == 64 * 512 + 1
    assert np.abs(a - b).max() < 1e-15
    from mmla_audio_amd.audio_segment import kaiser_best_table
    c, nc = kaiser_best_table()
    assert nc == 512 and np.array_equal(a, c)


@pytest.mark.parametrize('sr0,sr1', [(16000, 22050), (22050, 16000), (48000, 22050), (16000, 8000)])
def test_resampler_restatement_on_tones(sr0, sr1):
    """sanity of the (unpinned) resampy restatement: band-limited tones come out as the same tones.
    Downsampling is looser: resampy steps through the filter table by int(scale * 512) entries per
    tap while placing the first tap at the exact fraction -- the truncation detunes the outer taps a
    little (~-68 dB here), and the restatement keeps that."""
    t = np.arange(sr0) / sr0
    f = [440.0, 1800.0, 3000.0]
    x = sum(0.2 * np.sin(2 * np.pi * fk * t) for fk in f).astype(np.float32)
    y = ors.librosa_resample(x, sr0, sr1)
    assert len(y) == int(np.ceil(len(x) * sr1 / sr0))
    t1 = np.arange(len(y)) / sr1
    ref = sum(0.2 * np.sin(2 * np.pi * fk * t1) for fk in f)
    assert np.abs(y[400:-400] - ref[400:-400]).max() < (2e-6 if sr1 > sr0 else 1e-3)


def test_rms_long_full_scale_matches_audioop():
    """audioop.rms sums x*x in a float64 running sum, sample by sample; past 2^53 (~8.4 M
    full-scale samples) that sum rounds, so an exact integer sum gives a different (unsigned) rms
    for a long constant signal (32767 vs audioop's 32766 at 12 M samples)."""
    from mmla_audio_amd.audio_segment import AudioSegment
    for v, n in ((32767, 12_000_000), (30001, 16_000_000), (-32768, 9_000_000)):
        x = np.full(n, v, np.int16)
        assert AudioSegment(x, 16000).rms == audioop.rms(x.tobytes(), 2), (v, n)
    rng = np.random.default_rng(5)
    x = _pcm(rng, 10_000_000)
    assert AudioSegment(x, 16000).rms == audioop.rms(x.tobytes(), 2)
