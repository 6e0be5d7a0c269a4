"""Drop-in for ``noisereduce.reduce_noise(..., stationary=True)`` on the GPU.

The reference calls ``nr.reduce_noise(y_noise=noise, y=y, sr=sr, stationary=True)`` on float32
audio from ``librosa.load`` (``OverlapDetection/scripts/record_on_pc.py:208-212``,
``SpeakerIdentification/scripts/record_on_pc.py:189``,
``speaker_identification_post_processing.py:171``, ``record_on_pi.py:112``); ``import
mmla_audio_amd.noisereduce as nr`` keeps those lines unchanged.  The gate is noisereduce 2.0.x's
stationary spectral gate with its defaults (nr.hip; numerics in oracle/noisereduce.py).  Only the
stationary mode with default parameters is built; anything else raises, there is no CPU fallback.
"""
import numpy as np

from . import _lib

def _set_noise(ctx, y_noise, sr):
    """(Re)compute the noise profile on the device when the noise clip changes."""
    key = (hash(y_noise.tobytes()), y_noise.size, int(sr))
    if ctx.__dict__.get('_nr_key') != key:
        ctx.nr_set_noise(y_noise, sr)
        ctx._nr_key = key


def reduce_noise(y, sr, stationary=False, y_noise=None, prop_decrease=1.0, time_constant_s=2.0,
                 freq_mask_smooth_hz=500, time_mask_smooth_ms=50, thresh_n_mult_nonstationary=2,
                 sigmoid_slope_nonstationary=10, n_std_thresh_stationary=1.5, tmp_folder=None,
                 chunk_size=600000, padding=30000, n_fft=1024, win_length=None, hop_length=None,
                 clip_noise_stationary=True, use_tqdm=False, n_jobs=1, device=0):
    """noisereduce.reduce_noise (2.0.x signature).  y: [n] or [channels, n] float audio."""
    if not stationary:
        raise NotImplementedError('only stationary=True (the reference\'s call) is built')
    if (prop_decrease != 1.0 or freq_mask_smooth_hz != 500 or time_mask_smooth_ms != 50 or
            n_std_thresh_stationary != 1.5 or chunk_size != 600000 or padding != 30000 or
            n_fft != 1024 or win_length not in (None, 1024) or hop_length not in (None, 256) or
            not clip_noise_stationary):
        raise NotImplementedError('the GPU gate is built for noisereduce 2.0 defaults')
    y = np.asarray(y)
    dtype = y.dtype
    yn = np.asarray(y if y_noise is None else y_noise, dtype=np.float32)
    if yn.ndim > 1:                       # (channels, frames) -> one channel (SpectralGateStationary)
        yn = yn.mean(axis=0, dtype=np.float32)
    ctx = _lib.default_context(device)
    _set_noise(ctx, yn, sr)
    out = ctx.nr_reduce(np.atleast_2d(y).astype(np.float32))
    return (out[0] if y.ndim == 1 else out).astype(dtype)
