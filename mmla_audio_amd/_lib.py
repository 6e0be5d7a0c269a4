"""ctypes binding of libmmla.so (include/mmla.h).  The only way the Python side reaches the GPU.

There is deliberately no CPU fallback: if the in-tree ``libmmla.so`` is missing or no HIP device is
present, every entry point raises.  (The numpy restatement in ``oracle/`` is test infrastructure and
is never imported from here.)
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libmmla.so')

MMLA_OK = 0
MMLA_DEVICE_PTR = 0x1
MODEL_OD, MODEL_SI = 0, 1
HEAD_SOFTMAX, HEAD_SIGMOID = 0, 1
PREC_F32, PREC_F16X3 = 0, 1

OD_MELS, OD_FRAMES, OD_CLIP = 128, 151, 24000
SI_FRAMES, SI_DIMS, SI_SILENT_LEN = 256, 39, 4000

MMLA_E_RANGE = -6
_ERRORS = {-1: 'MMLA_E_INVALID', -2: 'MMLA_E_HIP', -3: 'MMLA_E_NOWEIGHTS', -4: 'MMLA_E_OOM',
           -5: 'MMLA_E_SHAPE', -6: 'MMLA_E_RANGE'}

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_U32 = ctypes.c_uint32

# name -> argtypes (all return int)
SIGNATURES = {
    'mmla_nr_set_noise': [_P, _P, _I64, ctypes.c_int32, ctypes.c_uint32],
    'mmla_nr_reduce': [_P, _P, _I64, _I64, _I64, _P, ctypes.c_uint32],
    'mmla_abi_version': [],
    'mmla_crc32c': [_P, _I64, ctypes.POINTER(_U32)],
    'mmla_png_unfilter': [_P, _I64, _I64, _I32, _P],
    'mmla_create': [ctypes.c_int, ctypes.POINTER(_P)],
    'mmla_destroy': [_P],
    'mmla_set_stream': [_P, _P],
    'mmla_synchronize': [_P],
    'mmla_set_microbatch': [_P, _I64, _I64],
    'mmla_get_microbatch': [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
    'mmla_release_workspace': [_P],
    'mmla_range_check': [_P, ctypes.POINTER(_I64)],
    'mmla_set_precision': [_P, ctypes.c_int],
    'mmla_load_weights': [_P, ctypes.c_int, _P, _I64, _I32, _I32],
    'mmla_od_features': [_P, _P, _I64, _I64, _P, _I32, _P, _P, _P, _P, _U32],
    'mmla_od_features_f32': [_P, _P, _I64, _I64, _P, _I32, _P, _P, _P, _P, _U32],
    'mmla_si_features': [_P, _P, _I64, _I64, _P, _I32, _P, _P, _U32],
    'mmla_si_features_seq': [_P, _P, _I64, _I64, _P, _U32],
    'mmla_od_forward': [_P, _P, _I64, _P, _U32],
    'mmla_od_forward_u8': [_P, _P, _I64, _P, _U32],
    'mmla_si_forward': [_P, _P, _I64, _P, _U32],
    'mmla_od_pipeline': [_P, _P, _I64, _I64, _P, _I32, _P, _P, _P, _U32],
    'mmla_si_pipeline': [_P, _P, _I64, _I64, _P, _I32, _P, _P, _P, _U32],
    'mmla_profile_enable': [_P, ctypes.c_int],
    'mmla_profile_read': [_P, _P, _P, _P, ctypes.c_int],
    'mmla_debug_od_trace': [_P, _P, _I64, ctypes.c_int, _P, _I64],
    'mmla_debug_ws_slot': [_P, ctypes.c_int, _P, _P],
    'mmla_debug_counters': [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
    'mmla_vad_reset': [_P, _I64, _I32],
    'mmla_vad_remove_silence': [_P, _P, _I64, _I64, _P, _I32, _I64, _P, _P, _P, _I32, _U32],
    'mmla_vad_collect': [_P, _P, _I64, _I64, _P, _I32, _P, _I32, _P, _P, _U32],
    'mmla_pcm16': [_P, _P, _I64, _P, _U32],
    'mmla_ratecv': [_P, _P, _I64, _I32, _I32, _I32, _P, _I64, _U32],
    'mmla_resample_sinc': [_P, _P, _I64, _I32, _I32, _P, _I64, _I32, _P, _I64, _U32],
}

NSTAGES = 7
STAGES = ('od_fe', 'si_fe', 'conv', 'lstm', 'glue', 'head', 'nr')

_lib = None
_lock = threading.Lock()


def load_library(path=LIB_PATH):
    """dlopen libmmla.so (raises OSError with a build hint if it is absent)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise OSError(f'{path} not found: build it with `make -C {os.path.join(_HERE, "csrc")}` '
                          f'or `python -c "import __graft_entry__ as g; g.build()"`')
        # PyTorch-ROCm ships its own libamdhip64.so.7 / libhsa-runtime64 (same sonames as
        # /opt/rocm's).  The first one loaded serves the whole process; torch cannot initialise on
        # /opt/rocm's newer runtime, while this library runs on torch's.  So when torch is present,
        # load it first: callers may then mix libmmla and torch device buffers in either order.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(path)
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        lib.mmla_last_error.argtypes = [_P]
        lib.mmla_last_error.restype = ctypes.c_char_p
        _lib = lib
        return lib


def crc32c(data):
    """CRC-32C of a bytes-like object (mmla_crc32c; host only, no device needed)."""
    lib = load_library()
    buf = np.frombuffer(memoryview(data).cast('B'), np.uint8)
    out = _U32()
    rc = lib.mmla_crc32c(buf.ctypes.data if buf.size else None, buf.size, ctypes.byref(out))
    if rc != MMLA_OK:
        raise MmlaError(f'mmla_crc32c: {_ERRORS.get(rc, rc)}', rc)
    return out.value


def png_unfilter(raw, h, row_bytes, bpp):
    """PNG scanline reconstruction (mmla_png_unfilter; host only, no device needed): the inflated
    IDAT bytes of h rows -> uint8 [h, row_bytes]."""
    lib = load_library()
    buf = np.frombuffer(memoryview(raw).cast('B'), np.uint8)
    if buf.size != h * (row_bytes + 1):
        raise ValueError(f'PNG image data holds {buf.size} bytes, expected {h} rows of '
                         f'{row_bytes + 1}')
    out = np.empty((h, row_bytes), np.uint8)
    rc = lib.mmla_png_unfilter(buf.ctypes.data if buf.size else None, h, row_bytes, bpp,
                               out.ctypes.data if out.size else None)
    if rc != MMLA_OK:
        raise ValueError('PNG image data: unknown scanline filter type')
    return out


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, int):
        return a
    return a.ctypes.data


class MmlaError(RuntimeError):
    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


class Context:
    """One libmmla context = one HIP device + stream + workspaces + loaded weights.

    Host-array methods take/return numpy arrays (synchronous).  ``*_dev`` methods take raw device
    pointers (ints, e.g. ``torch_tensor.data_ptr()``) and only enqueue on the context stream.
    """

    def __init__(self, device=0):
        self.lib = load_library()
        h = _P()
        rc = self.lib.mmla_create(int(device), ctypes.byref(h))
        if rc != MMLA_OK:
            raise MmlaError(f'mmla_create(device={device}) failed: {_ERRORS.get(rc, rc)} '
                            '(no HIP device visible?)')
        self.h = h
        self.device = device
        self.od_classes = None
        self.si_classes = None

    def close(self):
        if getattr(self, 'h', None):
            self.lib.mmla_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != MMLA_OK:
            msg = self.lib.mmla_last_error(self.h)
            raise MmlaError(f'{what}: {_ERRORS.get(rc, rc)}: {msg.decode() if msg else ""}', rc)

    # -- configuration ------------------------------------------------------------------------
    def set_stream(self, stream_handle):
        self._check(self.lib.mmla_set_stream(self.h, stream_handle), 'mmla_set_stream')

    def synchronize(self):
        self._check(self.lib.mmla_synchronize(self.h), 'mmla_synchronize')

    def set_precision(self, mode):
        """PREC_F16X3 (default, 3xFP16 MFMA convs) or PREC_F32 (exact f32 MFMA convs)."""
        self._check(self.lib.mmla_set_precision(self.h, int(mode)), 'mmla_set_precision')

    def set_microbatch(self, od=0, si=0):
        self._check(self.lib.mmla_set_microbatch(self.h, int(od), int(si)), 'mmla_set_microbatch')

    def get_microbatch(self):
        """-> (od_clips, si_clips) per internal micro-batch for the next call."""
        od, si = _I64(), _I64()
        self._check(self.lib.mmla_get_microbatch(self.h, ctypes.byref(od), ctypes.byref(si)),
                    'mmla_get_microbatch')
        return od.value, si.value

    def release_workspace(self):
        self._check(self.lib.mmla_release_workspace(self.h), 'mmla_release_workspace')

    def range_check(self):
        """Wait for the stream; -> number of host-call micro-batches re-run in exact f32 so far.
        Raises MmlaError (code MMLA_E_RANGE) if a device-pointer call overflowed the fp16 range."""
        n = _I64()
        self._check(self.lib.mmla_range_check(self.h, ctypes.byref(n)), 'mmla_range_check')
        return n.value

    def debug_counters(self):
        """-> (host micro-batches re-run in exact f32, host micro-batches re-run on the unsplit
        BiLSTM after a split-BiLSTM timeout) so far"""
        a, b = _I64(), _I64()
        self._check(self.lib.mmla_debug_counters(self.h, ctypes.byref(a), ctypes.byref(b)),
                    'mmla_debug_counters')
        return a.value, b.value

    def profile_enable(self, on=True):
        self._check(self.lib.mmla_profile_enable(self.h, int(bool(on))), 'mmla_profile_enable')

    def profile_read(self, reset=True):
        """-> {stage: (device ms, launches, algorithmic work)} accumulated since the last reset."""
        ms = np.zeros(NSTAGES, np.float64)
        n = np.zeros(NSTAGES, np.int64)
        wk = np.zeros(NSTAGES, np.float64)
        self._check(self.lib.mmla_profile_read(self.h, _ptr(ms), _ptr(n), _ptr(wk), int(reset)),
                    'mmla_profile_read')
        return {s: (float(ms[i]), int(n[i]), float(wk[i])) for i, s in enumerate(STAGES)}

    def debug_od_trace(self, x, stage):
        """OD-NET intermediate tensor after `stage` (see mmla.h) for float NHWC input x."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        n = x.shape[0]
        shapes = {0: (128, 151, 16), 10: (19, 128), 11: (512,)}
        hw = [(64, 76, 32), (64, 76, 32), (64, 76, 32), (32, 38, 64), (32, 38, 64), (32, 38, 64),
              (16, 19, 128), (16, 19, 128), (16, 19, 128)]
        shape = shapes.get(stage) or hw[stage - 1]
        out = np.empty((n,) + shape, np.float32)
        self._check(self.lib.mmla_debug_od_trace(self.h, _ptr(x), n, int(stage), _ptr(out), out.size),
                    'mmla_debug_od_trace')
        return out

    def load_weights(self, kind, packed, n_classes, head=HEAD_SOFTMAX):
        packed = np.ascontiguousarray(packed, dtype=np.float32)
        self._check(self.lib.mmla_load_weights(self.h, int(kind), _ptr(packed), packed.size,
                                               int(n_classes), int(head)), 'mmla_load_weights')
        if kind == MODEL_OD:
            self.od_classes = int(n_classes)
        else:
            self.si_classes = int(n_classes)

    # -- noise gate --------------------------------------------------------
    def nr_set_noise(self, noise, sr=16000):
        """Noise profile for reduce_noise(y_noise=noise, stationary=True): float32 samples."""
        a = np.ascontiguousarray(noise, dtype=np.float32).ravel()
        self._check(self.lib.mmla_nr_set_noise(self.h, _ptr(a), a.size, int(sr), 0),
                    'mmla_nr_set_noise')

    def nr_reduce(self, y):
        """Gate float32 signals y [n, len] (or [len]) with the current noise profile."""
        a = np.ascontiguousarray(y, dtype=np.float32)
        flat = a.ndim == 1
        if flat:
            a = a[None]
        out = np.empty_like(a)
        self._check(self.lib.mmla_nr_reduce(self.h, _ptr(a), a.shape[0], a.shape[1], a.shape[1],
                                            _ptr(out), 0), 'mmla_nr_reduce')
        return out[0] if flat else out

    def nr_reduce_dev(self, y, n, stride, length, out):
        self._check(self.lib.mmla_nr_reduce(self.h, y, n, stride, length, out, MMLA_DEVICE_PTR),
                    'mmla_nr_reduce(dev)')

    # -- silence removal -----------------------------------------------------
    def vad_reset(self, n_streams=1, mode=3):
        """n_streams fresh webrtcvad.Vad(mode) detectors (state kept in the context)."""
        self._check(self.lib.mmla_vad_reset(self.h, int(n_streams), int(mode)), 'mmla_vad_reset')
        self.vad_streams = int(n_streams)
        # whoever tagged the detector before (post-processing _vad_owner) no longer owns it
        self.vad_owner = None

    def vad_remove_silence(self, pcm, lens=None, items_per_stream=1):
        """save_wave_file(silence_remove=True) of every item: int16 [n, L] (or a list) ->
        (voiced PCM list of int16 arrays, per-frame speech flags list).  Items of one stream are
        consecutive and processed in order with that stream's detector state."""
        a, ln, L = self._pcm(pcm, lens)
        n = a.shape[0]
        nf = max(1, (a.shape[1] - 1) // 480) if a.shape[1] > 480 else 1
        out = np.empty_like(a)
        olen = np.empty(n, np.int32)
        sp = np.zeros((n, nf), np.uint8)
        self._check(self.lib.mmla_vad_remove_silence(
            self.h, _ptr(a), n, a.shape[1], _ptr(ln), L, int(items_per_stream), _ptr(out),
            _ptr(olen), _ptr(sp), nf, 0), 'mmla_vad_remove_silence')
        lens_in = ln if ln is not None else np.full(n, L, np.int32)
        nfr = [(int(m) - 1) // 480 if m > 480 else 0 for m in lens_in]
        return [out[i, :olen[i]].copy() for i in range(n)], [sp[i, :nfr[i]].astype(bool) for i in range(n)]

    def vad_collect(self, pcm, speech, lens=None):
        """the collector + rewrite alone on given per-frame decisions (list of bool arrays)"""
        a, ln, L = self._pcm(pcm, lens)
        n = a.shape[0]
        nf = max([1] + [len(s) for s in speech])
        sp = np.zeros((n, nf), np.uint8)
        for i, s in enumerate(speech):
            sp[i, :len(s)] = np.asarray(s, np.uint8)
        out = np.empty_like(a)
        olen = np.empty(n, np.int32)
        self._check(self.lib.mmla_vad_collect(self.h, _ptr(a), n, a.shape[1], _ptr(ln), L, _ptr(sp),
                                              nf, _ptr(out), _ptr(olen), 0), 'mmla_vad_collect')
        return [out[i, :olen[i]].copy() for i in range(n)]

    def pcm16(self, y):
        """float audio -> int16 as soundfile writes PCM_16"""
        a = np.ascontiguousarray(y, dtype=np.float32)
        out = np.empty(a.shape, np.int16)
        self._check(self.lib.mmla_pcm16(self.h, _ptr(a), a.size, _ptr(out), 0), 'mmla_pcm16')
        return out

    # -- rate conversion (offline pre-conditioning) ---------------------------------------------
    @staticmethod
    def ratecv_frames(n_frames, inrate, outrate):
        """output frames of audioop.ratecv(..., state=None) on n_frames input frames"""
        from math import gcd
        g = gcd(int(inrate), int(outrate))
        return (int(n_frames) - 1) * (int(outrate) // g) // (int(inrate) // g) + 1 if n_frames > 0 else 0

    def ratecv(self, pcm, nchannels, inrate, outrate):
        """audioop.ratecv(pcm, 2, nchannels, inrate, outrate, None)[0] (pydub set_frame_rate) on
        interleaved int16 frames -> int16 [out_frames * nchannels]"""
        a = np.ascontiguousarray(pcm, dtype=np.int16).reshape(-1)
        if a.size % nchannels:
            raise MmlaError(f'{a.size} samples are not whole frames of {nchannels} channels')
        nf = a.size // nchannels
        m = self.ratecv_frames(nf, inrate, outrate)
        out = np.empty(m * nchannels, np.int16)
        self._check(self.lib.mmla_ratecv(self.h, _ptr(a), nf, int(nchannels), int(inrate), int(outrate),
                                         _ptr(out), m, 0), 'mmla_ratecv')
        return out

    def resample_sinc(self, x, sr_orig, sr_new, half_window, num_table):
        """resampy.resample(x, sr_orig, sr_new, filter=(half_window, num_table)) on float32 mono"""
        a = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
        w = np.ascontiguousarray(half_window, dtype=np.float64)
        m = int(a.size * (float(sr_new) / sr_orig))
        out = np.empty(m, np.float32)
        self._check(self.lib.mmla_resample_sinc(self.h, _ptr(a), a.size, int(sr_orig), int(sr_new),
                                                _ptr(w), w.size, int(num_table), _ptr(out), m, 0),
                    'mmla_resample_sinc')
        return out

    # -- host-array API -----------------------------------------------------------------------
    @staticmethod
    def _pcm(pcm, lens):
        """-> (contiguous int16 [n, L], lens int32 [n] or None, clip_len)."""
        if isinstance(pcm, (list, tuple)):
            n = len(pcm)
            L = max([len(p) for p in pcm] + [1])
            buf = np.zeros((n, L), np.int16)
            ln = np.zeros(n, np.int32)
            for i, p in enumerate(pcm):
                buf[i, :len(p)] = np.asarray(p, np.int16)
                ln[i] = len(p)
            return buf, ln, L
        a = np.ascontiguousarray(pcm, dtype=np.int16)
        if a.ndim == 1:
            a = a[None]
        ln = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        return a, ln, a.shape[1]

    @staticmethod
    def _float_pcm(pcm, lens):
        """float audio (librosa.load scale: any floating dtype, or a list of float arrays) ->
        (contiguous float32 [n, L], lens int32 [n] or None, clip_len); None for integer PCM"""
        if isinstance(pcm, (list, tuple)):
            if not any(np.issubdtype(np.asarray(p).dtype, np.floating) for p in pcm):
                return None
            n = len(pcm)
            L = max([len(p) for p in pcm] + [1])
            buf = np.zeros((n, L), np.float32)
            ln = np.zeros(n, np.int32)
            for i, p in enumerate(pcm):
                buf[i, :len(p)] = np.asarray(p, np.float32)
                ln[i] = len(p)
            return buf, ln, L
        a = np.asarray(pcm)
        if not np.issubdtype(a.dtype, np.floating):
            return None
        a = np.ascontiguousarray(a, dtype=np.float32)
        if a.ndim == 1:
            a = a[None]
        ln = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        return a, ln, a.shape[1]

    def od_features(self, pcm, lens=None, db=True, norm=True, zcr=True, img=True):
        """int16 PCM [n, L] (or a list of 1-D int16 arrays) -> dict of features.  Float audio
        (librosa.load scale, any floating dtype or a list of float arrays) goes through
        mmla_od_features_f32 instead."""
        fl = self._float_pcm(pcm, lens)
        if fl is not None:
            a, ln, L = fl
            fn = self.lib.mmla_od_features_f32
        else:
            a, ln, L = self._pcm(pcm, lens)
            fn = self.lib.mmla_od_features
        n = a.shape[0]
        out = {}
        bufs = {}
        for key, want, shape, dt in (('db', db, (n, OD_MELS, OD_FRAMES), np.float32),
                                     ('norm', norm, (n, OD_MELS, OD_FRAMES), np.float32),
                                     ('zcr', zcr, (n, OD_FRAMES), np.float32),
                                     ('img', img, (n, OD_MELS, OD_FRAMES, 3), np.uint8)):
            bufs[key] = np.empty(shape, dt) if want else None
        self._check(fn(
            self.h, _ptr(a), n, a.shape[1], _ptr(ln), L, _ptr(bufs['db']), _ptr(bufs['norm']),
            _ptr(bufs['zcr']), _ptr(bufs['img']), 0), 'mmla_od_features')
        for k, v in bufs.items():
            if v is not None:
                out[k] = v
        return out

    def si_features(self, pcm, lens=None):
        a, ln, L = self._pcm(pcm, lens)
        n = a.shape[0]
        feat = np.empty((n, SI_FRAMES, SI_DIMS), np.float32)
        silent = np.empty(n, np.uint8)
        self._check(self.lib.mmla_si_features(self.h, _ptr(a), n, a.shape[1], _ptr(ln), L,
                                              _ptr(feat), _ptr(silent), 0), 'mmla_si_features')
        return feat, silent.astype(bool)

    def si_features_seq(self, sig):
        """Whole-signal features cut into 256-frame windows -> float32 [S, 256, 39]."""
        sig = np.ascontiguousarray(sig, dtype=np.int16).ravel()
        n = sig.size
        T = 1 if n <= 400 else 1 + -(-(n - 400) // 160)
        S = -(-T // SI_FRAMES)
        feat = np.empty((S, SI_FRAMES, SI_DIMS), np.float32)
        self._check(self.lib.mmla_si_features_seq(self.h, _ptr(sig), n, S, _ptr(feat), 0),
                    'mmla_si_features_seq')
        return feat

    def od_forward(self, x):
        x = np.ascontiguousarray(x)
        n = x.shape[0]
        probs = np.empty((n, 2), np.float32)
        if x.dtype == np.uint8:
            rc = self.lib.mmla_od_forward_u8(self.h, _ptr(x), n, _ptr(probs), 0)
        else:
            x = np.ascontiguousarray(x, dtype=np.float32)
            rc = self.lib.mmla_od_forward(self.h, _ptr(x), n, _ptr(probs), 0)
        self._check(rc, 'mmla_od_forward')
        return probs

    def si_forward(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        n = x.shape[0]
        probs = np.empty((n, self.si_classes or 0), np.float32)
        self._check(self.lib.mmla_si_forward(self.h, _ptr(x), n, _ptr(probs), 0), 'mmla_si_forward')
        return probs

    def od_pipeline(self, pcm, lens=None):
        """-> (probs [n,2], argmax [n] (-1 = 'silent'), silent [n] bool)."""
        a, ln, L = self._pcm(pcm, lens)
        n = a.shape[0]
        probs = np.empty((n, 2), np.float32)
        am = np.empty(n, np.int32)
        silent = np.empty(n, np.uint8)
        self._check(self.lib.mmla_od_pipeline(self.h, _ptr(a), n, a.shape[1], _ptr(ln), L,
                                              _ptr(probs), _ptr(am), _ptr(silent), 0),
                    'mmla_od_pipeline')
        return probs, am, silent.astype(bool)

    def od_pipeline_strided(self, signal, n, stride, clip_len):
        """OD pipeline over n windows of one long int16 signal: window c = signal[c*stride :
        c*stride + clip_len] (overlapping when stride < clip_len; no host-side copies)."""
        sig = np.ascontiguousarray(signal, dtype=np.int16).reshape(-1)
        if n < 0 or (n > 0 and (n - 1) * stride + clip_len > sig.size):
            raise MmlaError(f'{n} windows of {clip_len} at stride {stride} exceed {sig.size} samples')
        probs = np.empty((n, 2), np.float32)
        am = np.empty(n, np.int32)
        self._check(self.lib.mmla_od_pipeline(self.h, _ptr(sig), n, stride, None, clip_len,
                                              _ptr(probs), _ptr(am), None, 0), 'mmla_od_pipeline')
        return probs, am

    def od_features_strided(self, signal, n, stride, clip_len, db=True, norm=True, zcr=True, img=True):
        """OD features of n windows of one long signal: window c = signal[c*stride : c*stride +
        clip_len] (int16 -> mmla_od_features, float -> mmla_od_features_f32; no host copies)"""
        fl = np.issubdtype(np.asarray(signal).dtype, np.floating)
        sig = np.ascontiguousarray(signal, dtype=np.float32 if fl else np.int16).reshape(-1)
        if n < 0 or (n > 0 and (n - 1) * stride + clip_len > sig.size):
            raise MmlaError(f'{n} windows of {clip_len} at stride {stride} exceed {sig.size} samples')
        bufs = {}
        for key, want, shape, dt in (('db', db, (n, OD_MELS, OD_FRAMES), np.float32),
                                     ('norm', norm, (n, OD_MELS, OD_FRAMES), np.float32),
                                     ('zcr', zcr, (n, OD_FRAMES), np.float32),
                                     ('img', img, (n, OD_MELS, OD_FRAMES, 3), np.uint8)):
            bufs[key] = np.empty(shape, dt) if want else None
        fn = self.lib.mmla_od_features_f32 if fl else self.lib.mmla_od_features
        self._check(fn(self.h, _ptr(sig), n, stride, None, clip_len, _ptr(bufs['db']),
                       _ptr(bufs['norm']), _ptr(bufs['zcr']), _ptr(bufs['img']), 0),
                    'mmla_od_features(strided)')
        return {k: v for k, v in bufs.items() if v is not None}

    def si_pipeline(self, pcm, lens=None):
        a, ln, L = self._pcm(pcm, lens)
        n = a.shape[0]
        probs = np.empty((n, self.si_classes or 0), np.float32)
        am = np.empty(n, np.int32)
        silent = np.empty(n, np.uint8)
        self._check(self.lib.mmla_si_pipeline(self.h, _ptr(a), n, a.shape[1], _ptr(ln), L,
                                              _ptr(probs), _ptr(am), _ptr(silent), 0),
                    'mmla_si_pipeline')
        return probs, am, silent.astype(bool)

    # -- device-pointer API (asynchronous on the context stream) -------------------------------
    def od_features_dev(self, pcm, n, stride, clip_len, db=0, norm=0, zcr=0, img=0, lens=0):
        self._check(self.lib.mmla_od_features(self.h, pcm, n, stride, lens or None, clip_len,
                                              db or None, norm or None, zcr or None, img or None,
                                              MMLA_DEVICE_PTR), 'mmla_od_features(dev)')

    def si_features_dev(self, pcm, n, stride, clip_len, feat, silent=0, lens=0):
        self._check(self.lib.mmla_si_features(self.h, pcm, n, stride, lens or None, clip_len, feat,
                                              silent or None, MMLA_DEVICE_PTR),
                    'mmla_si_features(dev)')

    def od_pipeline_dev(self, pcm, n, stride, clip_len, probs=0, argmax=0, lens=0, silent=0):
        self._check(self.lib.mmla_od_pipeline(self.h, pcm, n, stride, lens or None, clip_len,
                                              probs or None, argmax or None, silent or None,
                                              MMLA_DEVICE_PTR),
                    'mmla_od_pipeline(dev)')

    def si_pipeline_dev(self, pcm, n, stride, clip_len, probs=0, argmax=0, silent=0, lens=0):
        self._check(self.lib.mmla_si_pipeline(self.h, pcm, n, stride, lens or None, clip_len,
                                              probs or None, argmax or None, silent or None,
                                              MMLA_DEVICE_PTR), 'mmla_si_pipeline(dev)')

    def od_forward_dev(self, x, n, probs, u8=False):
        fn = self.lib.mmla_od_forward_u8 if u8 else self.lib.mmla_od_forward
        self._check(fn(self.h, x, n, probs, MMLA_DEVICE_PTR), 'mmla_od_forward(dev)')

    def si_forward_dev(self, x, n, probs):
        self._check(self.lib.mmla_si_forward(self.h, x, n, probs, MMLA_DEVICE_PTR),
                    'mmla_si_forward(dev)')


_default = {}


def default_context(device=None):
    """Process-wide context per device (device defaults to LOCAL_RANK or 0)."""
    if device is None:
        device = int(os.environ.get('LOCAL_RANK', 0))
    if device not in _default:
        _default[device] = Context(device)
    return _default[device]
