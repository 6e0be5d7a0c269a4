"""The slice of pydub and librosa.load that the reference's offline pre-conditioning calls.

``standardize_audio`` in both offline scripts (OverlapDetection/scripts/
overlap_detection_post_processing.py:101-148, SpeakerIdentification/scripts/
speaker_identification_post_processing.py:136-188) goes through

* ``AudioSegment.from_file(path, format)`` / ``.set_frame_rate(16000)`` / ``.dBFS`` /
  ``.apply_gain(db)`` / ``.export(path, format='wav')`` (pydub), and
* ``librosa.load(path)`` at its DEFAULT rate 22050 (SI :142; librosa 0.8 resamples with resampy's
  ``kaiser_best`` filter) and ``librosa.load(path, sr=None)``.

``AudioSegment`` keeps pydub's semantics for 16-bit WAV data of any channel count and rate:
``set_frame_rate`` is ``audioop.ratecv(data, 2, channels, rate, new_rate, None)`` and runs on the
GPU (mmla_ratecv, resample.hip; bit-identical to CPython's audioop, tests/test_gpu_resample.py);
``dBFS`` is pydub's ``20 * math.log(audioop.rms / 2^15, 10)`` and ``apply_gain`` ``audioop.mul(data, 2,
10^(db/20))`` (host arithmetic, pinned against stdlib audioop in tests/test_resample_cpu.py).
``load`` is librosa.load(path, sr=22050 | None, mono=True) for WAV files; its resampling step is
resampy's sinc interpolation on the GPU (mmla_resample_sinc) with the ``kaiser_best`` filter built
here -- resampy is not installed in this image, so that step's parity is unpinned.
"""
import math
import wave

import numpy as np

from . import _lib

# resampy 0.2 'kaiser_best': Kaiser-windowed sinc, 64 zero crossings, 2^9 samples per crossing
KAISER_BEST = dict(num_zeros=64, precision=9, beta=14.769656459379492, rolloff=0.9475937167399596)


def kaiser_best_table():
    """resampy.filters.sinc_window(num_zeros=64, precision=9, window=kaiser(beta), rolloff) ->
    (right half of the interpolated filter, float64 [64 * 512 + 1], samples per zero crossing)"""
    p = KAISER_BEST
    num_bits = 2 ** p['precision']
    n = num_bits * p['num_zeros']
    sinc_win = p['rolloff'] * np.sinc(p['rolloff'] * np.linspace(0, p['num_zeros'], num=n + 1,
                                                                   endpoint=True))
    taper = np.kaiser(2 * n + 1, p['beta'])[n:]
    return taper * sinc_win, num_bits


_TABLE = {}


def resample(y, orig_sr, target_sr, ctx=None):
    """librosa 0.8 ``resample(y, orig_sr, target_sr, res_type='kaiser_best', fix=True)`` of float32
    mono audio: resampy's sinc interpolation (GPU), then fix_length to ceil(n * ratio)."""
    y = np.ascontiguousarray(y, dtype=np.float32).reshape(-1)
    if orig_sr == target_sr:
        return y
    ctx = ctx or _lib.default_context()
    if 'kb' not in _TABLE:
        _TABLE['kb'] = kaiser_best_table()
    win, num_table = _TABLE['kb']
    n_samples = int(np.ceil(y.shape[-1] * float(target_sr) / orig_sr))
    y_hat = ctx.resample_sinc(y, orig_sr, target_sr, win, num_table)
    if len(y_hat) < n_samples:
        y_hat = np.pad(y_hat, (0, n_samples - len(y_hat)))
    return np.ascontiguousarray(y_hat[:n_samples], dtype=np.float32)


def _read_wav(path):
    """(rate, channels, sample width, interleaved samples) of a PCM WAV file"""
    with wave.open(path, 'rb') as f:
        nch, width, rate, n = f.getparams()[:4]
        data = f.readframes(n)
    if width == 2:
        x = np.frombuffer(data, dtype='<i2').astype(np.int16)
    elif width == 4:
        x = np.frombuffer(data, dtype='<i4').astype(np.int32)
    elif width == 1:
        x = np.frombuffer(data, dtype=np.uint8).copy()
    else:
        raise ValueError(f'{path}: {8 * width}-bit WAV data is not supported')
    return rate, nch, width, x


def load(path, sr=22050, mono=True, ctx=None):
    """``librosa.load(path, sr=sr, mono=True)`` for WAV files -> (float32 y, sr).  soundfile's
    float32 scaling (16-bit x / 2^15, 32-bit x / 2^31, unsigned 8-bit (x - 128) / 2^7), the float32
    channel mean, then -- unless sr is None or the file's rate -- the kaiser_best resampling."""
    if not mono:
        raise ValueError('only mono=True (the reference never asks for more)')
    rate, nch, width, x = _read_wav(path)
    if width == 2:
        y = x.astype(np.float32) / np.float32(32768.0)
    elif width == 4:
        y = x.astype(np.float32) * np.float32(2.0 ** -31)
    else:
        y = (x.astype(np.float32) - np.float32(128.0)) * np.float32(1.0 / 128.0)
    if nch > 1:
        y = np.mean(y.reshape(-1, nch).T, axis=0)        # librosa.to_mono
    y = np.ascontiguousarray(y, dtype=np.float32)
    if sr is not None and sr != rate:
        y = resample(y, rate, sr, ctx)
        rate = sr
    return y, rate


class AudioSegment:
    """pydub.AudioSegment for 16-bit PCM WAV data (what the reference's recordings and zoom
    exports are): ``data`` int16 interleaved frames."""

    sample_width = 2

    def __init__(self, data, frame_rate, channels=1, ctx=None):
        self.data = np.ascontiguousarray(data, dtype=np.int16).reshape(-1)
        if self.data.size % channels:
            raise ValueError(f'{self.data.size} samples are not whole {channels}-channel frames')
        self.frame_rate = int(frame_rate)
        self.channels = int(channels)
        self._ctx = ctx

    @classmethod
    def from_file(cls, path, format=None, ctx=None):
        rate, nch, width, x = _read_wav(path)
        if width != 2:
            raise ValueError(f'{path}: {8 * width}-bit WAV; the GPU ratecv is built for 16-bit PCM')
        return cls(x, rate, nch, ctx)

    from_wav = from_file

    @property
    def ctx(self):
        return self._ctx or _lib.default_context()

    def _spawn(self, data, frame_rate=None):
        return AudioSegment(data, frame_rate or self.frame_rate, self.channels, self._ctx)

    def __len__(self):
        """duration in ms, as pydub"""
        return round(1000 * (self.data.size // self.channels) / self.frame_rate)

    @property
    def frame_count(self):
        return self.data.size // self.channels

    def get_array_of_samples(self):
        return self.data.copy()

    def set_frame_rate(self, frame_rate):
        """audioop.ratecv(data, 2, channels, rate, frame_rate, None) on the GPU"""
        if frame_rate == self.frame_rate:
            return self
        if self.data.size == 0:
            return self._spawn(self.data, frame_rate)
        out = self.ctx.ratecv(self.data, self.channels, self.frame_rate, frame_rate)
        return self._spawn(out, frame_rate)

    @property
    def rms(self):
        """audioop.rms(data, 2): (unsigned int) sqrt(sum(x^2) / n) with a float64 running sum,
        accumulated sample by sample in order as CPython's loop does (np.add.accumulate is that
        sequential loop; np.sum's pairwise sum and an exact int64 sum differ from it once the sum
        passes 2^53, i.e. after ~8.4 M full-scale samples).  Chunks of 2^20 samples carry the running
        sum, so memory stays O(chunk) for hour-long files with the same summation order."""
        if self.data.size == 0:
            return 0
        flat = self.data.reshape(-1)
        total = 0.0
        for i in range(0, flat.size, 1 << 20):
            c = flat[i:i + (1 << 20)].astype(np.float64)
            total = float(np.add.accumulate(np.concatenate(([total], c * c)))[-1])
        return int(np.sqrt(total / self.data.size))

    max_possible_amplitude = 2 ** 15

    @property
    def dBFS(self):
        """pydub: ratio_to_db(rms / max_possible_amplitude) = 20 * math.log(ratio, 10) (pydub's own
        expression: math.log with a base is log(x) / log(10), which can differ from log10 in the
        last bit); -inf for silence"""
        rms = self.rms
        if not rms:
            return -float('inf')
        return 20 * math.log(rms / float(self.max_possible_amplitude), 10)

    def apply_gain(self, volume_change):
        """audioop.mul(data, 2, 10 ** (volume_change / 20)): per sample x * factor in double,
        bounded (> 32767 -> 32767, < -32767 -> -32768) and floored"""
        factor = 10.0 ** (float(volume_change) / 20.0)
        return self._spawn(mul(self.data, factor))

    def export(self, out_f, format='wav'):
        if format not in (None, 'wav'):
            raise ValueError(f'export format {format!r}: only wav')
        with wave.open(out_f, 'wb') as f:
            f.setnchannels(self.channels)
            f.setsampwidth(2)
            f.setframerate(self.frame_rate)
            f.writeframes(self.data.astype('<i2').tobytes())
        return out_f


def mul(pcm, factor):
    """audioop.mul(pcm, 2, factor) on int16 samples"""
    v = np.asarray(pcm, dtype=np.float64) * float(factor)
    v = np.where(v > 32767.0, 32767.0, np.where(v < -32767.0, -32768.0, v))
    return np.floor(v).astype(np.int16)


def rms(pcm):
    return AudioSegment(pcm, 16000).rms
