"""Stationary noise-reduction oracle (numpy/scipy) -- TEST INFRASTRUCTURE ONLY, never product code.

Restates ``nr.reduce_noise(y_noise=noise, y=y, sr=sr, stationary=True)`` as the reference calls it
(``OverlapDetection/scripts/record_on_pc.py:208-212``,
``SpeakerIdentification/scripts/record_on_pc.py:189``,
``speaker_identification_post_processing.py:171``, ``record_on_pi.py:112``).  ``noisereduce`` is
unpinned in ``setup.py:32``; the keyword call ``reduce_noise(y=, sr=, y_noise=, stationary=)`` is the
2.x API, and the numpy==1.21 / librosa-0.8 era of the repo makes that noisereduce 2.0.x, whose
stationary gate runs on librosa's ``stft`` / ``istft`` / ``amplitude_to_db``.  Neither noisereduce
nor librosa is installed here and no reference-held vector covers this path: parity is *unpinned*;
this file restates their published 2.0.x / 0.8.x algorithms:

  * defaults: n_fft 1024, win_length = n_fft, hop = win_length // 4, n_std_thresh_stationary 1.5,
    prop_decrease 1.0, freq_mask_smooth_hz 500, time_mask_smooth_ms 50, chunk_size 600 000,
    padding 30 000, clip_noise_stationary True;
  * noise profile: STFT of ``y_noise[:chunk_size]`` (float32 -> complex64, as librosa.load gives
    float32), ``amplitude_to_db(|X|, ref=1, amin=1e-20, top_db=80)`` in float32, threshold per bin
    = mean + 1.5 std over frames (float32);
  * signal: every chunk is read into a float64 buffer with ``padding`` samples of context on both
    sides (zeros outside the signal), STFT (complex128), dB (top_db relative to the chunk's
    maximum), mask = dB > threshold, mask smoothed by ``fftconvolve(mask, filter, 'same')`` with the
    outer product of triangular ramps (33 bins x 7 frames at 16 kHz), STFT x mask, ``istft``
    (window-sum-square normalised, centre trimmed), the chunk's interior kept, cast to float32.
"""
import numpy as np
from scipy.signal import fftconvolve

N_FFT = 1024
HOP = 256
N_STD = 1.5
CHUNK = 600000
PADDING = 30000


def hann(n=N_FFT):
    """scipy.signal.get_window('hann', n, fftbins=True): periodic Hann, float64."""
    k = np.arange(n)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def stft(y, n_fft=N_FFT, hop=HOP):
    """librosa 0.8 stft(y, n_fft, hop_length, win_length=n_fft, window='hann', center=True,
    pad_mode='reflect'): [1 + n_fft/2, frames], complex64 for float32 y, complex128 for float64."""
    out_dtype = np.complex64 if y.dtype == np.float32 else np.complex128
    yp = np.pad(y, n_fft // 2, mode='reflect')
    n_frames = 1 + (len(yp) - n_fft) // hop
    idx = np.arange(n_fft)[:, None] + hop * np.arange(n_frames)[None, :]
    frames = yp[idx] * hann(n_fft)[:, None]            # float64 (float64 window)
    return np.fft.rfft(frames, axis=0).astype(out_dtype)


def window_sumsquare(n_frames, n_fft=N_FFT, hop=HOP):
    """librosa.filters.window_sumsquare(window='hann', n_frames, win_length=n_fft, n_fft, hop)."""
    n = n_fft + hop * (n_frames - 1)
    x = np.zeros(n)
    w2 = hann(n_fft) ** 2
    for i in range(n_frames):
        s = i * hop
        x[s:min(n, s + n_fft)] += w2[:max(0, min(n_fft, n - s))]
    return x


def istft(S, n_fft=N_FFT, hop=HOP):
    """librosa 0.8 istft(S, hop_length, win_length=n_fft, window='hann', center=True, length=None):
    overlap-add of windowed irfft frames, divided by the window sum-square where it is > tiny,
    n_fft / 2 trimmed from both ends.  float64 for complex128 input."""
    n_frames = S.shape[1]
    frames = np.fft.irfft(S, n=n_fft, axis=0) * hann(n_fft)[:, None]
    y = np.zeros(n_fft + hop * (n_frames - 1))
    for t in range(n_frames):
        y[t * hop: t * hop + n_fft] += frames[:, t]
    wss = window_sumsquare(n_frames, n_fft, hop)
    nz = wss > np.finfo(wss.dtype).tiny
    y[nz] /= wss[nz]
    return y[n_fft // 2: -(n_fft // 2)]


def amp_to_db(x, amin=1e-20, top_db=80.0):
    """noisereduce _amp_to_db = librosa.amplitude_to_db(x, ref=1.0, amin=1e-20, top_db=80.0),
    computed in x's dtype (float32 for the noise profile, float64 for the signal)."""
    mag = np.abs(x)
    power = np.square(mag)
    log_spec = 10.0 * np.log10(np.maximum(amin ** 2, power))
    log_spec = log_spec - 10.0 * np.log10(np.maximum(amin ** 2, 1.0))
    return np.maximum(log_spec, log_spec.max() - top_db)


def smoothing_filter(n_grad_freq, n_grad_time):
    """noisereduce _smoothing_filter: outer product of triangular ramps, normalised to sum 1."""
    f = np.concatenate([np.linspace(0, 1, n_grad_freq + 1, endpoint=False),
                        np.linspace(1, 0, n_grad_freq + 2)])[1:-1]
    t = np.concatenate([np.linspace(0, 1, n_grad_time + 1, endpoint=False),
                        np.linspace(1, 0, n_grad_time + 2)])[1:-1]
    s = np.outer(f, t)
    return s / np.sum(s)


def grads(sr, n_fft=N_FFT, hop=HOP, freq_mask_smooth_hz=500, time_mask_smooth_ms=50):
    """(n_grad_freq, n_grad_time) of SpectralGate._generate_mask_smoothing_filter: (16, 3) at 16 kHz."""
    return (int(freq_mask_smooth_hz / (sr / (n_fft / 2))),
            int(time_mask_smooth_ms / ((hop / sr) * 1000)))


def noise_threshold(y_noise, n_fft=N_FFT, hop=HOP, n_std=N_STD, chunk=CHUNK):
    """SpectralGateStationary.__init__: per-bin threshold (float32) from the noise clip."""
    yn = np.asarray(y_noise, dtype=np.float32)[:chunk]
    db = amp_to_db(np.abs(stft(yn, n_fft, hop)))          # float32 [bins, frames]
    mean = np.mean(db, axis=1)
    std = np.std(db, axis=1)
    return (mean + std * np.float32(n_std)).astype(np.float32)


def gate_chunk(chunk, thresh, sr, n_fft=N_FFT, hop=HOP, prop_decrease=1.0):
    """spectral_gating_stationary on one float64 chunk."""
    S = stft(chunk, n_fft, hop)
    db = amp_to_db(np.abs(S))
    mask = db > thresh[:, None]
    mask = mask * prop_decrease + np.ones(np.shape(mask)) * (1.0 - prop_decrease)
    mask = fftconvolve(mask, smoothing_filter(*grads(sr, n_fft, hop)), mode='same')
    y = istft(S * mask, n_fft, hop)
    out = np.zeros(chunk.shape)
    out[:len(y)] = y
    return out


def reduce_noise(y, sr, y_noise, n_fft=N_FFT, hop=HOP, chunk_size=CHUNK, padding=PADDING,
                 prop_decrease=1.0, n_std=N_STD):
    """reduce_noise(y=y, sr=sr, y_noise=y_noise, stationary=True) for a mono float32 y."""
    y = np.asarray(y)
    dtype = y.dtype
    n = len(y)
    thresh = noise_threshold(y_noise, n_fft, hop, n_std, chunk_size)

    def filter_chunk(start, end):
        i1, i2 = start - padding, end + padding
        buf = np.zeros(i2 - i1)
        a, b = max(i1, 0), min(i2, n)
        buf[a - i1:b - i1] = y[a:b]
        return gate_chunk(buf, thresh, sr, n_fft, hop, prop_decrease)[start - i1:end - i1]

    if n > chunk_size:     # SpectralGate.get_traces: chunk by chunk, each with its padding context
        out = np.zeros(n)
        for i in range(int((n - 1) / chunk_size) + 1):
            s, e = i * chunk_size, min((i + 1) * chunk_size, n)
            out[s:e] = filter_chunk(i * chunk_size, (i + 1) * chunk_size)[:e - s]
        return out.astype(dtype)
    return filter_chunk(0, n).astype(dtype)
