"""Why the SI front-end keeps its FFT in float64 ("prove the choice with a
committed worst-case clip").

python_speech_features frames without a window (rectangular, `numpy.ones`), so leakage puts energy in
every band and speech-like clips are benign: a float32 FFT stays near 3e-6 of the float64 features.
The worst case is a loud tone just below Nyquist: pre-emphasis boosts it, the low bands then hold
only leakage many decades down, and the float32 round-off of the frame (relative to its total
energy) dominates their log energies -- at 7980 Hz full scale the float32-FFT features miss the
float64 reference by 2.4e-4, over the 1e-4 bar.  The float64 FFT keeps such clips at the
1e-6 level (tests/test_gpu_parity.py::test_si_features_worst_case_tones runs them through the
kernel).  The float32 variant here only replaces the FFT of the oracle (speaker_identification.py:386
-> psf.mfcc -> powspec); everything else stays the float64 restatement.
"""
import numpy as np
import pytest

from oracle import si_fe, synth

WORST_TONES = (7950, 7980)   # Hz, full scale, 1.5 s


def tone(f, n=24000, amp=32767):
    t = np.arange(n) / 16000.0
    return np.round(amp * np.sin(2 * np.pi * f * t)).astype(np.int16)


def features_fft32(pcm):
    """the oracle's 39 features with the rFFT computed in float32 (numpy >= 2 keeps the precision)"""
    orig = si_fe.powspec

    def powspec32(frames, nfft=si_fe.NFFT):
        x = np.fft.rfft(frames.astype(np.float32), nfft)
        assert x.dtype == np.complex64
        return 1.0 / nfft * np.square(np.absolute(x.astype(np.complex128)))

    si_fe.powspec = powspec32
    try:
        return si_fe.features_39(pcm)
    finally:
        si_fe.powspec = orig


@pytest.mark.parametrize('f', WORST_TONES)
def test_float32_fft_misses_the_bar_on_near_nyquist_tones(f):
    p = tone(f)
    err = np.abs(features_fft32(p) - si_fe.features_39(p)).max()
    assert err > 1e-4, f'{f} Hz: float32-FFT error {err:.3g} -- the worst case is no longer one'


def test_float32_fft_is_benign_on_speech_like_clips():
    worst = max(np.abs(features_fft32(synth.clip(i, 24000)) - si_fe.features_39(synth.clip(i, 24000))).max()
                for i in range(5))
    assert worst < 1e-5
