"""Drop-in for ``OverlapDetection/scripts/overlap_features_generator.py`` (class OverlapFeaturesGenerator).

Same names, arguments and return values as the reference (``:29-151``); the arithmetic runs in the
``od_fe`` HIP kernel through ``libmmla.so``.  A caller switches with one import line::

    from mmla_audio_amd.overlap_features_generator import OverlapFeaturesGenerator

Batched entry point (no PNG on the hot path): ``OverlapFeaturesGenerator.generate_batch(pcm)``.
"""
import os
import struct
import zlib

import numpy as np
import scipy.io.wavfile as _wavfile

from . import _lib


def _load(path):
    """``librosa.load(path, sr=None)`` (mono=True; overlap_features_generator.py:72,93) for WAV files.

    librosa 0.8 reads through soundfile as float32 (16-bit x / 2^15, 32- and left-justified 24-bit
    x / 2^31, unsigned 8-bit (x - 128) / 2^7, float files as stored) and downmixes with the channel
    mean (``to_mono``: np.mean over channels in float32).  A 16-bit mono file is returned as its
    int16 samples (the kernel applies / 32768 itself, exactly); anything else as that float32
    signal, which the float entry point (mmla_od_features_f32) consumes.

    ``sr=None`` keeps the file's rate and the reference then builds its mel basis and FFT framing
    from it; the HIP front-end is built for 16 kHz only, so any other rate raises ValueError
    instead of silently computing a 16 kHz spectrogram."""
    sr, x = _wavfile.read(path)
    if sr != 16000:
        raise ValueError(f'{path}: sample rate {sr} Hz; the HIP front-end computes the reference\'s '
                         'features at 16 kHz only (librosa.load(sr=None) keeps the file rate)')
    if x.dtype == np.int16 and x.ndim == 1:
        return sr, x
    if x.dtype == np.int16:
        y = x.astype(np.float32) / np.float32(32768.0)
    elif x.dtype == np.int32:
        y = x.astype(np.float32) * np.float32(2.0 ** -31)
    elif x.dtype == np.uint8:
        y = (x.astype(np.float32) - np.float32(128.0)) * np.float32(1.0 / 128.0)
    elif x.dtype in (np.float32, np.float64):
        y = x.astype(np.float32)
    else:
        raise ValueError(f'{path}: unsupported WAV sample type {x.dtype}')
    if y.ndim > 1:
        y = np.mean(y.T, axis=0)          # librosa.to_mono on [channels, n]
    return sr, np.ascontiguousarray(y, dtype=np.float32)


def _features(ctx, x, **kw):
    return ctx.od_features(x[None], lens=np.array([len(x)], np.int32), **kw)


def write_png_rgba(path, rgb):
    """Write the image file ``plt.imsave(path, img, origin="lower")`` writes (:151) for the already
    flipped and quantised uint8 pixels ``rgb``: through matplotlib's own writer when it is
    importable (uint8 RGB is written as is, alpha 255 -- the same bytes as the reference for the
    same pixels and matplotlib version), else a minimal RGBA PNG encoder.  Either way decoders
    reading 3 channels (``tf.image.decode_png(img, 3)``, record_on_pc.py:157) get ``rgb`` back."""
    try:
        from matplotlib import image as mimage
    except ImportError:
        mimage = None
    if mimage is not None:
        mimage.imsave(path, np.ascontiguousarray(rgb, dtype=np.uint8), origin='upper')
        return
    h, w, _ = rgb.shape
    rgba = np.empty((h, w, 4), np.uint8)
    rgba[..., :3] = rgb
    rgba[..., 3] = 255
    raw = b''.join(b'\x00' + rgba[r].tobytes() for r in range(h))

    def chunk(tag, data):
        c = struct.pack('>I', len(data)) + tag + data
        return c + struct.pack('>I', zlib.crc32(tag + data) & 0xFFFFFFFF)

    png = b'\x89PNG\r\n\x1a\n' + chunk(b'IHDR', struct.pack('>IIBBBBB', w, h, 8, 6, 0, 0, 0))
    png += chunk(b'IDAT', zlib.compress(raw, 6)) + chunk(b'IEND', b'')
    with open(path, 'wb') as f:
        f.write(png)


class OverlapFeaturesGenerator:
    """overlap_features_generator.py:29-151 on the GPU."""

    def __init__(self, wl, hl, sr=16000, device=None):
        self.sr = sr
        self.window_length = int(sr * (wl / 1000))
        self.hop_length = int(sr * (hl / 1000))
        self.time_dim = 150
        self.mel_dim = 128
        if (self.window_length, self.hop_length, sr) != (400, 160, 16000):
            raise ValueError('the HIP front-end is built for wl=25 ms, hl=10 ms at 16 kHz, the only '
                             'configuration the reference uses (record_on_pc.py:85)')
        self._device = device

    @property
    def _ctx(self):
        return _lib.default_context(self._device)

    def get_attributes(self):
        return self.window_length, self.hop_length, self.sr

    def resize_mel_features(self, features_arr):
        """overlap_features_generator.py:51-63 (host-side, unchanged semantics)."""
        if features_arr.shape[1] < self.time_dim:
            pad = self.time_dim - features_arr.shape[1]
            features_arr = np.pad(features_arr, ((0, 0), (0, pad)), 'constant')
        return features_arr[:self.mel_dim, :self.time_dim]

    # -- per-file API (reference signatures) ----------------------------------------------------
    def generate_mels(self, wav_file_path, n_mels=128):
        """-> (s_db float32 [128,151], s_db_norm float32 [128,151])  (:65-85)."""
        if n_mels != 128:
            raise ValueError('n_mels must be 128 (the kernel is built for the reference default)')
        _, x = _load(wav_file_path)
        f = _features(self._ctx, x, zcr=False, img=False)
        return f['db'][0], f['norm'][0]

    def generate_zcr(self, wav_file_path):
        """-> float64 [1, 151] zero-crossing rate (:87-101)."""
        _, x = _load(wav_file_path)
        f = _features(self._ctx, x, db=False, norm=False, img=False)
        return self._zcr64(f['zcr'][0])[None]

    @staticmethod
    def _zcr64(z32):
        # the kernel's float32 count/400 -> the reference's float64 count/400, exactly
        return np.rint(z32.astype(np.float64) * 400.0) / 400.0

    @staticmethod
    def normalize_matrix(m):
        """(:103-117) min-max normalisation with float32 scalar semantics (NaN if constant)."""
        m = np.asarray(m)
        max_val = np.max(m)
        min_val = np.min(m)
        diff = max_val - min_val
        with np.errstate(invalid='ignore', divide='ignore'):
            return ((m - min_val) / diff).astype(m.dtype)

    def generate_zcr_image(self, wav_file_path, out_dir, out_name=None):
        """(:133-151).  out_name None -> float64 [128,151,3] image (R = zcr, G = B = 1 - norm);
        otherwise writes ``out_dir + out_name`` as the PNG the reference's plt.imsave writes."""
        if not os.path.isdir(out_dir):
            os.mkdir(out_dir)
        _, x = _load(wav_file_path)
        f = _features(self._ctx, x, db=False)
        if out_name is None:
            img = np.empty((128, 151, 3), np.float64)
            img[..., 0] = self._zcr64(f['zcr'][0])[None, :]
            g = 1.0 - f['norm'][0].astype(np.float64)
            img[..., 1] = g
            img[..., 2] = g
            return img
        write_png_rgba(out_dir + out_name, f['img'][0])
        return None

    # -- batched API (the MI355X-native path) ----------------------------------------------------
    def generate_batch(self, pcm, lens=None, db=False, norm=True, zcr=True, img=True):
        """int16 PCM [n, L] (or a list of 1-D arrays) -> dict of batched features."""
        return self._ctx.od_features(pcm, lens=lens, db=db, norm=norm, zcr=zcr, img=img)
