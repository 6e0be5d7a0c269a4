"""Drop-in for the feature functions of ``SpeakerIdentification/scripts/speaker_identification.py``.

``input_feature_gen`` (:372-398) and ``delta`` (:141-151) keep their names and return values;
the MFCC / delta / delta-delta / pad-to-256 path runs in the ``si_fe`` HIP kernel (float64 math).
``make_feature_experiment`` (:317-369), used by the registration/transfer-learning callers, keeps
its chunked output layout.
"""
import math
import os
import sys
import time

import numpy as np
import scipy.io.wavfile as _wavfile

from . import _lib


def delta(feat, N):
    """speaker_identification.py:141-151 (edge-padded regression delta), vectorised on the host.
    Exposed for API compatibility; the batched GPU path computes deltas inside the kernel."""
    feat = np.asarray(feat)
    denominator = 2 * sum([i ** 2 for i in range(1, N + 1)])
    padded = np.pad(feat, ((N, N), (0, 0)), mode='edge')
    t = len(feat)
    out = np.zeros_like(feat, dtype=np.result_type(feat.dtype, np.float64))
    for n in range(-N, N + 1):
        if n:
            out = out + n * padded[N + n:N + n + t]
    return (out / denominator).astype(np.result_type(feat.dtype, np.float64))


def _read(path):
    rate, sig = _wavfile.read(path)
    if rate != 16000:
        raise ValueError(f'{path}: the HIP MFCC is built for 16 kHz, got {rate}')
    if sig.dtype != np.int16 or sig.ndim != 1:
        raise ValueError(f'{path}: expected mono int16 PCM')
    return sig


def input_feature_gen(wav_path, device=None):
    """-> 'silent' (fewer than 4000 samples) or float64 [1, 256, 39] (:372-398)."""
    sig = _read(wav_path)
    if len(sig) < _lib.SI_SILENT_LEN:
        return 'silent'
    feat, silent = _lib.default_context(device).si_features(sig[None], lens=np.array([len(sig)], np.int32))
    return feat.astype(np.float64)


def input_feature_batch(pcm, lens=None, device=None):
    """Batched input_feature_gen: int16 [n, L] (or list) -> (float32 [n, 256, 39], silent [n])."""
    return _lib.default_context(device).si_features(pcm, lens=lens)


_speakers_count_dict = {}   # the reference binarizer's mutable default argument: process-wide


def binarizer(str_list, dim, speakers_count_dict=_speakers_count_dict):
    """speaker_identification.py:122-138, same semantics: first-occurrence numbering that restarts
    at 0 on every call while the dict (a mutable default argument) keeps the labels of earlier
    calls -- so a new speaker in a later call can share an index with an old one, and an index
    >= dim raises IndexError, exactly as in the reference."""
    if not str_list:
        raise UnboundLocalError("local variable 'result' referenced before assignment")
    count = 0
    rows = np.zeros((len(str_list), dim))
    for i, s in enumerate(str_list):
        if s not in speakers_count_dict:
            speakers_count_dict[s] = count
            count += 1
        rows[i, speakers_count_dict[s]] = 1
    return rows


def make_feature_experiment(wav_files, device=None):
    """(:317-369): per file MFCC+deltas over the WHOLE file, zero-padded to a multiple of 256 frames
    and cut into 256-frame windows; labels = file stem; returns (x float64 [S,256,39], one-hot y,
    speaker_id dict) with the reference's binarizer (state kept across calls).  Whole-file features
    are produced chunk-aligned on the GPU (see conversation_features)."""
    train_x, train_y = [], []
    begin = time.time()
    for i, onewav in enumerate(wav_files):
        if i % 5 == 4:
            gap = time.time() - begin
            sys.stdout.write('\r%.2f %% used:%ds' % (float(i) * 100 / len(wav_files), gap))
        label = os.path.basename(onewav)[:-4]
        chunks = conversation_features(_read(onewav), device=device)
        for c in chunks:
            train_x.append(c)
            train_y.append(label)
    y = binarizer(train_y, dim=len(set(train_y)))
    speaker_id = {str(int(np.argmax(y[i]))): train_y[i] for i in range(len(train_y))}
    return np.asarray(train_x), y, speaker_id


def conversation_features(sig, device=None):
    """Whole-sequence MFCC + deltas cut into 256-frame windows -> float64 [S, 256, 39]
    (speaker_identification_post_processing.py:255-269; make_feature_experiment :341-353)."""
    return _lib.default_context(device).si_features_seq(np.asarray(sig, np.int16)).astype(np.float64)
