"""OverlapDetection front-end oracle (numpy) -- TEST INFRASTRUCTURE ONLY, never product code.

Restates, operation by operation and dtype by dtype, what the reference computes in
``OverlapFeaturesGenerator.generate_mels / generate_zcr / generate_zcr_image``
(``OverlapDetection/scripts/overlap_features_generator.py:65-151``) on top of
librosa 0.8.x, numpy 1.21 and matplotlib.  librosa is not installed in this image, so the
librosa parts below are restatements of its published 0.8.x source (pinned version in
SURVEY.md section 8c): parity of those parts is *unpinned* by any reference-held vector.

dtype notes (numpy 1.21 value-based casting, which the reference ran under, ``setup.py:32-35``):
  * ``stft``: periodic Hann (float64) * float32 frames -> float64 rFFT -> stored complex64.
  * ``np.abs(complex64) ** 2`` -> float32 (hypotf, then square).
  * mel basis built in float64, stored float32, Slaney-normalised in a float64 loop -> float32.
  * ``power_to_db(ref=np.max)``: the per-element log is float32; the reference term
    ``10*log10(max(1e-10, np.float32 max))`` is a *scalar-scalar* op and therefore float64 under
    numpy 1.x, then cast to float32 when subtracted from the float32 array.
  * ``normalize_matrix``: float32 scalars (``overlap_features_generator.py:110-116``).
  * image G/B = ``1 - np.float32`` -> float64 under numpy 1.x; R = count/400 float64;
    ``plt.imsave`` quantises with ``(v * 255).astype(uint8)`` in float64 and flips rows
    (``origin="lower"``).
"""
import numpy as np

SR = 16000
N_FFT = 400          # int(16000 * 25 / 1000)  overlap_features_generator.py:39
HOP = 160            # int(16000 * 10 / 1000)  overlap_features_generator.py:40
TIME_DIM = 150       # overlap_features_generator.py:41
N_MELS = 128         # overlap_features_generator.py:42 / generate_mels default
CLIP = HOP * TIME_DIM            # 24000 samples: pad/trunc length, :73-80
N_FRAMES = 1 + CLIP // HOP       # 151 (center=True)
N_BINS = 1 + N_FFT // 2          # 201


def load_int16(pcm):
    """librosa.load(path, sr=None) on a 16-bit mono WAV: soundfile float32 = x / 32768.  A float32
    array is taken as librosa.load's output already (any other WAV format, stereo downmixed)."""
    pcm = np.asarray(pcm)
    if pcm.dtype == np.float32:
        return pcm
    return (pcm.astype(np.int16).astype(np.float32) / np.float32(32768.0)).astype(np.float32)


def pad_trunc(y, n=CLIP):
    """overlap_features_generator.py:73-80 (and :94-98): zero-pad to n, then keep y[:n]."""
    y = np.asarray(y, dtype=np.float32)
    if len(y) < n:
        y = np.pad(y, (0, n - len(y)), 'constant')
    return y[:n]


def hann_periodic(n=N_FFT):
    """scipy.signal.get_window('hann', n, fftbins=True) -> float64."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def frame(y, frame_length, hop_length):
    n = 1 + (len(y) - frame_length) // hop_length
    idx = np.arange(frame_length)[:, None] + hop_length * np.arange(n)[None, :]
    return y[idx]   # [frame_length, n_frames] (librosa.util.frame layout)


def stft_power(y, n_fft=N_FFT, hop_length=HOP):
    """librosa 0.8 ``_spectrogram`` (power=2) via ``stft(center=True, pad_mode='reflect')``.

    Returns float32 [1 + n_fft//2, n_frames].
    """
    y = np.asarray(y, dtype=np.float32)
    win = hann_periodic(n_fft).reshape(-1, 1)                   # float64
    yp = np.pad(y, n_fft // 2, mode='reflect')
    frames = frame(yp, n_fft, hop_length)                        # float32
    spec = np.fft.rfft(win * frames, axis=0).astype(np.complex64)  # float64 FFT, complex64 store
    return (np.abs(spec) ** 2).astype(np.float32)


def _hz_to_mel_slaney(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if f.ndim:
        log_t = f >= min_log_hz
        mels = np.array(mels, dtype=np.float64)
        mels[log_t] = min_log_mel + np.log(f[log_t] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def _mel_to_hz_slaney(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    log_t = m >= min_log_mel
    freqs[log_t] = min_log_hz * np.exp(logstep * (m[log_t] - min_log_mel))
    return freqs


def mel_frequencies(n_mels=128, fmin=0.0, fmax=11025.0):
    """librosa.mel_frequencies (htk=False)."""
    mels = np.linspace(_hz_to_mel_slaney(fmin), _hz_to_mel_slaney(fmax), n_mels)
    return _mel_to_hz_slaney(mels)


def mel_basis(sr=SR, n_fft=N_FFT, n_mels=N_MELS):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin=0, fmax=sr/2, htk=False, norm='slaney',
    dtype=float32) -> float32 [n_mels, 1 + n_fft//2]."""
    fmax = float(sr) / 2
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.linspace(0, float(sr) / 2, 1 + n_fft // 2, endpoint=True)
    mel_f = mel_frequencies(n_mels + 2, fmin=0.0, fmax=fmax)
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))    # float64 -> float32 store
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]                             # float64 loop, float32 out
    return weights


def melspectrogram(y, sr=SR, hop_length=HOP, n_fft=N_FFT, n_mels=N_MELS):
    """librosa.feature.melspectrogram(y, sr, hop_length, n_fft, n_mels) -> float32 [n_mels, T]
    (overlap_features_generator.py:81)."""
    S = stft_power(y, n_fft=n_fft, hop_length=hop_length)
    return np.dot(mel_basis(sr, n_fft, n_mels), S)


def power_to_db(S, top_db=80.0, amin=1e-10):
    """librosa.power_to_db(S, ref=np.max) with numpy 1.21 promotion (overlap_features_generator.py:82)."""
    S = np.asarray(S, dtype=np.float32)
    log_spec = (np.float32(10.0) * np.log10(np.maximum(np.float32(amin), S))).astype(np.float32)
    ref_value = float(np.max(S))                                 # np.float32 scalar
    ref_db = 10.0 * np.log10(max(amin, ref_value))               # scalar-scalar: float64
    log_spec = (log_spec - np.float32(ref_db)).astype(np.float32)
    thr = np.float32(float(log_spec.max()) - top_db)             # float64 scalar -> f32 in maximum
    return np.maximum(log_spec, thr).astype(np.float32)


def normalize_matrix(m):
    """OverlapFeaturesGenerator.normalize_matrix (overlap_features_generator.py:103-117), vectorised,
    float32 scalar semantics.  A constant matrix gives diff == 0 -> NaN, exactly like the reference."""
    m = np.asarray(m, dtype=np.float32)
    max_val = np.float32(np.max(m))
    min_val = np.float32(np.min(m))
    diff = np.float32(max_val - min_val)
    with np.errstate(invalid='ignore', divide='ignore'):
        return ((m - min_val).astype(np.float32) / diff).astype(np.float32)


def zero_crossing_rate(y, frame_length=N_FFT, hop_length=HOP):
    """librosa.feature.zero_crossing_rate(y, frame_length, hop_length) (center=True, edge pad,
    threshold=1e-10, zero_pos=True, pad=False) -> float64 [1, T] (overlap_features_generator.py:100)."""
    y = np.asarray(y, dtype=np.float32)
    yp = np.pad(y, frame_length // 2, mode='edge')
    fr = frame(yp, frame_length, hop_length).copy()
    fr[np.abs(fr) <= 1e-10] = 0
    s = np.signbit(fr)
    cross = np.pad(s[:-1] != s[1:], [(1, 0), (0, 0)], mode='constant', constant_values=False)
    return np.mean(cross, axis=0, keepdims=True)


def generate_mels(pcm):
    """generate_mels (overlap_features_generator.py:65-85) on int16 PCM -> (s_db, s_db_norm)."""
    y = pad_trunc(load_int16(pcm))
    s = melspectrogram(y)
    s_db = power_to_db(s)
    return s_db, normalize_matrix(s_db)


def generate_zcr(pcm):
    """generate_zcr (overlap_features_generator.py:87-101) -> float64 [1, 151]."""
    return zero_crossing_rate(pad_trunc(load_int16(pcm)))


def zcr_image(norm, zcr):
    """generate_zcr_image assembly (overlap_features_generator.py:139-146) -> float64 [128,151,3]
    (R = zcr, G = B = 1 - norm; the 1 - np.float32 is float64 under numpy 1.x)."""
    img = np.empty(norm.shape + (3,), dtype=np.float64)
    img[..., 0] = np.asarray(zcr, dtype=np.float64)[0][None, :]
    g = 1.0 - norm.astype(np.float64)
    img[..., 1] = g
    img[..., 2] = g
    return img


def quantize_png(img):
    """plt.imsave(origin='lower') + decode_png(channels=3): rows reversed, uint8 = trunc(v*255)
    (record_on_pc.py:156-158).  NaN (digital silence) -> 0, the x86 cast result."""
    flipped = img[::-1]
    with np.errstate(invalid='ignore'):
        v = flipped * 255
    out = np.zeros(v.shape, dtype=np.uint8)
    ok = np.isfinite(v)
    out[ok] = v[ok].astype(np.uint8)
    return out


def od_features(pcm):
    """All OD-FE outputs for one clip of int16 PCM (any length; first 24 000 samples used)."""
    s_db, norm = generate_mels(pcm)
    zcr = generate_zcr(pcm)
    img = zcr_image(norm, zcr)
    return {
        'db': s_db,                        # float32 [128,151]
        'norm': norm,                      # float32 [128,151]
        'zcr': zcr,                        # float64 [1,151]
        'image': img,                      # float64 [128,151,3], not flipped
        'png_rgb': quantize_png(img),      # uint8 [128,151,3], model input order (flipped)
    }


def zcr_counts(pcm):
    """Integer crossing counts per frame (zcr * 400), used for bit-exact checks."""
    return np.rint(generate_zcr(pcm)[0] * N_FFT).astype(np.int32)
