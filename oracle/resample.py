"""Rate conversion used by the reference's offline pre-conditioning -- TEST INFRASTRUCTURE ONLY.

Two resamplers sit upstream of the features in the offline chains:

* pydub ``AudioSegment.set_frame_rate(16000)`` (OverlapDetection/scripts/
  overlap_detection_post_processing.py:120-121, SpeakerIdentification/scripts/
  speaker_identification_post_processing.py:159-160) is ``audioop.ratecv(data, width, channels,
  rate, 16000, None)``.  ``ratecv`` below restates CPython's ``audioop.ratecv`` (Modules/audioop.c,
  weightA = 1, weightB = 0, fresh state) in closed form; stdlib ``audioop`` is importable in this
  image, so the restatement is pinned against it bit for bit (tests/test_resample_cpu.py).
* ``librosa.load(path)`` at its default sr = 22050 (speaker_identification_post_processing.py:142)
  resamples with resampy's ``kaiser_best`` filter (librosa 0.8 ``resample(res_type='kaiser_best')``).
  resampy is NOT installed here and no reference-held vector covers it: ``resample_kaiser_best`` is a
  restatement of resampy 0.2's published ``sinc_window`` filter construction and ``resample_f`` loop,
  **parity unpinned**.
"""
import numpy as np

# resampy 0.2 'kaiser_best' (filters.py / the shipped kaiser_best.npz): a Kaiser-windowed sinc
KAISER_BEST = dict(num_zeros=64, precision=9, beta=14.769656459379492, rolloff=0.9475937167399596)


def ratecv_len(n_frames, inrate, outrate):
    """output frames of audioop.ratecv(..., state=None) on n_frames input frames"""
    from math import gcd
    g = gcd(inrate, outrate)
    inrate //= g
    outrate //= g
    if n_frames <= 0:
        return 0
    return (n_frames - 1) * outrate // inrate + 1


def ratecv(pcm, nchannels, inrate, outrate):
    """audioop.ratecv(pcm.tobytes(), 2, nchannels, inrate, outrate, None)[0] for int16 PCM
    (interleaved frames) -> int16 array.

    The C loop keeps a phase counter d (starting at -outrate): each input frame adds outrate, each
    output frame subtracts inrate.  Output frame j is therefore written after input frame
    k = ceil(j * inrate / outrate) was read, with d = k * outrate - j * inrate in [0, outrate), from
    prev = frame k - 1 (0 before the first) and cur = frame k, both scaled to 32 bits (x << 16):
        out = (int)((prev * d + cur * (outrate - d)) / outrate)   (double arithmetic)  >> 16."""
    from math import gcd
    x = np.asarray(pcm, dtype=np.int16).reshape(-1, nchannels)
    g = gcd(inrate, outrate)
    ir, orr = inrate // g, outrate // g
    n_out = ratecv_len(len(x), inrate, outrate)
    j = np.arange(n_out, dtype=np.int64)
    k = -((-j * ir) // orr)                      # ceil(j ir / or)
    d = (k * orr - j * ir).astype(np.float64)
    cur = x[k].astype(np.float64) * 65536.0
    prev = np.where((k > 0)[:, None], x[np.maximum(k - 1, 0)].astype(np.float64) * 65536.0, 0.0)
    v = (prev * d[:, None] + cur * (orr - d)[:, None]) / float(orr)
    iv = np.trunc(v).astype(np.int64)             # C (int) cast
    return (iv >> 16).astype(np.int16).reshape(-1)


def kaiser_best_table(window='numpy'):
    """resampy.filters.sinc_window(64, 9, kaiser(beta), rolloff) -> (interp_win float64, num_bits).
    resampy built its table with scipy's Kaiser window; numpy's (the same I0 formula, numpy's own
    Bessel routine) agrees to ~1e-16 and is what the drop-in uses, so window='numpy' gives the
    identical table for bit-level checks of the resampling loop."""
    import scipy.signal
    p = KAISER_BEST
    num_bits = 2 ** p['precision']
    n = num_bits * p['num_zeros']
    sinc_win = p['rolloff'] * np.sinc(p['rolloff'] * np.linspace(0, p['num_zeros'], num=n + 1,
                                                                   endpoint=True))
    if window == 'numpy':
        taper = np.kaiser(2 * n + 1, p['beta'])[n:]
    else:
        taper = scipy.signal.windows.kaiser(2 * n + 1, p['beta'])[n:]
    return taper * sinc_win, num_bits


def resample_out_len(n, sr_orig, sr_new):
    """resampy's output length int(n * sr_new / sr_orig) (librosa 0.8 then fix_length()s it to
    ceil(n * ratio))"""
    return int(n * (float(sr_new) / sr_orig))


def resample_kaiser_best(x, sr_orig, sr_new, table=None):
    """resampy.resample(x, sr_orig, sr_new, filter='kaiser_best') on float32 mono x -> float32,
    restating resampy 0.2 core.resample / resample_f: per output t, the left wing then the right
    wing of the interpolated filter, each tap added to a float32 accumulator (numba: float64 product,
    float32 store); the time register advances by repeated float64 addition."""
    x = np.asarray(x, dtype=np.float32)
    interp_win, num_table = table if table is not None else kaiser_best_table()
    interp_win = np.array(interp_win, dtype=np.float64)
    ratio = float(sr_new) / sr_orig
    n_out = resample_out_len(len(x), sr_orig, sr_new)
    if ratio < 1:
        interp_win = interp_win * ratio
    delta = np.zeros_like(interp_win)
    delta[:-1] = np.diff(interp_win)
    scale = min(1.0, ratio)
    inc = 1.0 / ratio
    index_step = int(scale * num_table)
    nwin = len(interp_win)
    n_orig = len(x)
    tr = np.zeros(n_out, np.float64)
    if n_out > 1:
        tr[1:] = np.cumsum(np.full(n_out - 1, inc))    # sequential float64 additions
    n = tr.astype(np.int64)
    y = np.zeros(n_out, np.float32)
    x64 = x.astype(np.float64)
    # left wing
    frac = scale * (tr - n)
    index_frac = frac * num_table
    offset = index_frac.astype(np.int64)
    eta = index_frac - offset
    i_max = np.minimum(n + 1, (nwin - offset) // index_step)
    for i in range(int(i_max.max(initial=0))):
        m = i < i_max
        o = offset[m] + i * index_step
        w = interp_win[o] + eta[m] * delta[o]
        y[m] = (y[m].astype(np.float64) + w * x64[n[m] - i]).astype(np.float32)
    # right wing
    frac = scale - frac
    index_frac = frac * num_table
    offset = index_frac.astype(np.int64)
    eta = index_frac - offset
    k_max = np.minimum(n_orig - n - 1, (nwin - offset) // index_step)
    for k in range(int(k_max.max(initial=0))):
        m = k < k_max
        o = offset[m] + k * index_step
        w = interp_win[o] + eta[m] * delta[o]
        y[m] = (y[m].astype(np.float64) + w * x64[n[m] + k + 1]).astype(np.float32)
    return y


def librosa_resample(y, orig_sr, target_sr, table=None):
    """librosa 0.8 resample(y, orig_sr, target_sr, res_type='kaiser_best', fix=True, scale=False)"""
    y = np.asarray(y, dtype=np.float32)
    if orig_sr == target_sr:
        return y
    n_samples = int(np.ceil(y.shape[-1] * float(target_sr) / orig_sr))
    y_hat = resample_kaiser_best(y, orig_sr, target_sr, table)
    if len(y_hat) < n_samples:
        y_hat = np.pad(y_hat, (0, n_samples - len(y_hat)))
    return np.ascontiguousarray(y_hat[:n_samples], dtype=np.float32)
