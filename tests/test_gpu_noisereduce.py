"""GPU stationary noise gate against the oracle restatement of noisereduce
2.0.x (oracle/noisereduce.py; parity with the real library is unpinned: it is not installed).

Tolerance: the gate is a threshold decision per (bin, frame); the GPU recomputes the float32 noise
statistics with a different summation order and log implementation, so a bin whose dB sits within
~1e-6 dB of its threshold may flip.  Outputs must agree to 1e-5 (relative to the signal's peak) on
>= 99.9 % of samples and to 2e-2 everywhere; on these signals no flip occurs in practice and the
measured error is ~1e-7.
"""
import numpy as np
import pytest

from oracle import noisereduce as onr
from oracle import synth

pytestmark = pytest.mark.gpu


def _signals():
    rng = np.random.default_rng(5)
    noise = (0.01 * rng.standard_normal(48000)).astype(np.float32)
    t = np.arange(40000) / 16000
    tone = (0.3 * np.sin(2 * np.pi * 440 * t) + 0.01 * rng.standard_normal(40000)).astype(np.float32)
    speech = (synth.clip(91, 40000).astype(np.float32) / 32768.0).astype(np.float32)
    pure = (0.01 * rng.standard_normal(40000)).astype(np.float32)
    return noise, np.stack([tone, speech, pure])


def _close(got, want):
    peak = np.abs(want).max() + 1e-12
    err = np.abs(got.astype(np.float64) - want) / peak
    assert np.quantile(err, 0.999) <= 1e-5 and err.max() <= 2e-2, (np.quantile(err, 0.999), err.max())
    return err.max()


def test_reduce_noise_matches_oracle():
    from mmla_audio_amd import noisereduce as nr
    noise, ys = _signals()
    for y in ys:
        got = nr.reduce_noise(y=y, sr=16000, y_noise=noise, stationary=True)
        want = onr.reduce_noise(y, 16000, noise)
        assert got.dtype == np.float32 and got.shape == y.shape
        _close(got, want)


def test_batched_equals_single():
    from mmla_audio_amd import _lib
    noise, ys = _signals()
    ctx = _lib.Context(0)
    ctx.nr_set_noise(noise)
    batch = ctx.nr_reduce(ys)
    for i, y in enumerate(ys):
        assert np.array_equal(batch[i], ctx.nr_reduce(y))


def test_long_signal_is_chunked_like_get_traces():
    from mmla_audio_amd import noisereduce as nr
    rng = np.random.default_rng(6)
    noise = (0.02 * rng.standard_normal(20000)).astype(np.float32)
    y = np.concatenate([synth.clip(100 + k, 40000) for k in range(16)]).astype(np.float32) / 32768
    y = (y[:620000] + 0.02 * rng.standard_normal(620000)).astype(np.float32)   # 2 chunks
    got = nr.reduce_noise(y=y, sr=16000, y_noise=noise, stationary=True)
    _close(got, onr.reduce_noise(y, 16000, noise))


def test_unsupported_modes_raise():
    from mmla_audio_amd import noisereduce as nr
    y = np.zeros(1000, np.float32)
    with pytest.raises(NotImplementedError):
        nr.reduce_noise(y=y, sr=16000, stationary=False)
    with pytest.raises(NotImplementedError):
        nr.reduce_noise(y=y, sr=16000, stationary=True, prop_decrease=0.5)


@pytest.mark.parametrize('n', [1, 10, 700, 1025, 5000])
def test_short_signals(n):
    """Signals shorter than one frame / a few frames: every window reaches the buffer's reflect
    edges' zero padding, and the launched frame range (nr_frame_range) is small."""
    from mmla_audio_amd import noisereduce as nr
    noise, ys = _signals()
    y = ys[1][:n].copy()
    got = nr.reduce_noise(y=y, sr=16000, y_noise=noise, stationary=True)
    _close(got, onr.reduce_noise(y, 16000, noise))


def test_silent_signal():
    """All-zero input: every frame is the -400 dB floor (the top_db reference of the chunk)."""
    from mmla_audio_amd import noisereduce as nr
    noise, _ = _signals()
    y = np.zeros(40000, np.float32)
    got = nr.reduce_noise(y=y, sr=16000, y_noise=noise, stationary=True)
    want = onr.reduce_noise(y, 16000, noise)
    assert np.array_equal(got, want.astype(np.float32))


def test_zero_run_inside_signal_after_other_calls():
    """A run of >= 1024 zero samples inside a voiced signal: its all-zero windows still reach the
    kept interior, so their spectra (0) are read by the gate; the scratch holding the previous
    call's spectra must not leak in (regression: the first call on a fresh context passed)."""
    from mmla_audio_amd import _lib
    noise, ys = _signals()
    ctx = _lib.Context(0)
    ctx.nr_set_noise(noise)
    ctx.nr_reduce(np.stack([ys[0], ys[1]]))                # fill the scratch with nonzero spectra
    y = ys[1].copy()
    y[9000:13800] = 0.0
    y[30000:31100] = 0.0
    got = ctx.nr_reduce(y)
    _close(got, onr.reduce_noise(y, 16000, noise))
