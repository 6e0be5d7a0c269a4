"""Offline OverlapDetection post-processing on the MI355X path.

Mirrors OverlapDetection/scripts/overlap_detection_post_processing.py:

* ``segmentation(src_dir, dst_dir, win_time_stride, step_time)`` (:23-85) -- cuts every WAV of a
  directory into fixed windows and writes them as ``<name>/<name>_<j>_<rate>_split.wav``; same
  segment count formula, same file names, byte-identical WAV files (tests/test_segmentation.py pins
  them against the reference's own output, tests/golden/seg_golden.npz).  One deliberate deviation:
  the reference joins ``src_dir + "\\" + f`` (a Windows separator, :33); this joins with
  ``os.path.join`` so it also runs on Linux.
* ``predict_segments(...)`` -- the per-segment loop of ``post_anlysing`` (:184-226: cut, write WAV,
  ``generate_zcr_image`` -> PNG -> ``decode_png`` -> ``model.predict`` -> argmax, batch 1 per
  segment) as ONE fused GPU call: the windows are strided views of the conversation PCM (no copies,
  overlapping when step < window), features and OD-NET run on the device.  ``write_log`` writes the
  reference's TSV log (:212-226) from the result.
* ``standardize_audio(...)`` (:101-148) and ``post_anlysing(root_dir, model)`` (:151-226): the whole
  offline chain -- standardise every conversation under ``experiment/recordings/post-time/whole``
  (dBFS gain, the stationary noise gate 3x for ``audio*`` files on nr.hip, PCM_16 rewrites),
  segment the standardised files (1.5 s / 1.5 s), ONE fused features + OD-NET call per
  conversation over its segment windows, and the TSV log per conversation with the segments in
  the order ``os.listdir`` returns them, as the reference's loop does.  Pinned against the
  reference's own post_anlysing run with stubs (tests/golden/odpost_golden.npz).
"""
import os
import wave
from datetime import datetime, timedelta

import numpy as np

OVERLAP_DEGREE = {'0': 'non-overlapped', '1': 'overlapped'}   # overlap_detection_post_processing.py:18
# the fused pipeline's argmax is -1 for a window shorter than 4000 samples (the 'silent' sentinel of
# record_on_pc.py:141-154); the reference's offline loop never sees one (1.5 s segments)
LABELS = dict(OVERLAP_DEGREE, **{'-1': 'silent'})


def segment_bounds(nframes, framerate, win_time_stride, step_time):
    """(window frames, step frames, segment count) exactly as the reference computes them (:50-53)."""
    win = int(framerate * win_time_stride)
    step = int(framerate * step_time)
    cut_num = int(((nframes - win) / step) + 1)
    return win, step, max(cut_num, 0)


def segmentation(src_dir, dst_dir, win_time_stride, step_time):
    """Cut the WAVs of ``src_dir`` into ``win_time_stride``-second windows every ``step_time``
    seconds, written under ``dst_dir/<name>/`` (overlap_detection_post_processing.py:23-85)."""
    files = [os.path.join(src_dir, f) for f in os.listdir(src_dir) if f.endswith('.wav')]
    for filename in files:
        with wave.open(filename, 'rb') as f:
            nchannels, sampwidth, framerate, nframes = f.getparams()[:4]
            str_data = f.readframes(nframes)
        wave_data = np.frombuffer(str_data, dtype=np.short)
        temp_data = wave_data.reshape(-1, 2) if nchannels > 1 else wave_data   # frames x channels

        win_num_frames, step_num_frames, cut_num = segment_bounds(nframes, framerate,
                                                                  win_time_stride, step_time)
        print("window frames: ", win_num_frames, "step frames: ", step_num_frames)
        step_total_num_frames = 0
        base = os.path.splitext(os.path.split(filename)[-1])[0]
        file_save_path = os.path.join(dst_dir, base)
        for j in range(cut_num):
            if not os.path.exists(file_save_path):
                os.makedirs(file_save_path)
            out_file = os.path.join(file_save_path, base + '_%d_%s_split.wav' % (j, framerate))
            start = step_num_frames * j
            seg = np.ascontiguousarray(temp_data[start:start + win_num_frames]).astype(np.short)
            step_total_num_frames = (j + 1) * step_num_frames
            with wave.open(out_file, 'wb') as f:
                f.setnchannels(nchannels)
                f.setsampwidth(sampwidth)
                f.setframerate(framerate)
                f.writeframes(seg.tobytes())
        print("Total number of frames :", nframes, " Extract frames: ", step_total_num_frames)


def predict_segments(pcm, model, sr=16000, win_time_stride=1.5, step_time=1.5):
    """All windows of one mono 16 kHz int16 conversation through the fused OD pipeline.

    Returns (probs float32 [n, 2], argmax int32 [n], labels list of 'overlapped'/'non-overlapped').
    ``model`` is an ``OverlapDetectionModel`` (``models.load_model``).
    """
    if sr != 16000:
        raise ValueError(f'the OD front-end is defined at 16 kHz (got {sr})')
    sig = np.ascontiguousarray(pcm, dtype=np.int16).reshape(-1)
    win, step, n = segment_bounds(sig.size, sr, win_time_stride, step_time)
    if n == 0:
        return np.zeros((0, 2), np.float32), np.zeros(0, np.int32), []
    model._ensure_loaded()
    probs, am = model.ctx.od_pipeline_strided(sig, n, step, win)
    return probs, am, [LABELS[str(int(k))] for k in am]


def predict_wav(path, model, win_time_stride=1.5, step_time=1.5):
    """``predict_segments`` of a mono int16 WAV file (the standardized conversation of :199)."""
    with wave.open(path, 'rb') as f:
        nchannels, sampwidth, framerate, nframes = f.getparams()[:4]
        if nchannels != 1 or sampwidth != 2:
            raise ValueError(f'{path}: expected mono int16, got {nchannels} ch x {8 * sampwidth} bit')
        sig = np.frombuffer(f.readframes(nframes), dtype=np.short)
    return predict_segments(sig, model, framerate, win_time_stride, step_time)


def write_log(log_path, argmax, start_time=None):
    """The per-conversation TSV log of post_anlysing (:212-226): a header, then one line per
    segment with its overlap degree and a timestamp advancing 1.5 s per segment (hard-coded there)."""
    time = start_time or datetime.today()
    with open(log_path, 'w') as f:
        f.write('segment' + '\t' + 'overlapped degree' + '\t' + 'timestamp')
        f.write('\n')
        for count, k in enumerate(argmax):
            if count > 0:
                time = time + timedelta(seconds=1.5)
            f.write(str(count) + '\t' + str(LABELS[str(int(k))]) + '\t' + str(time))
            f.write('\n')


# ---- the offline chain (post_anlysing) --------------------------------------------------------

def _read_pcm16(path):
    """(rate, int16 PCM) of a mono 16-bit WAV: what AudioSegment.from_file hands pydub for the
    reference's recordings.  Other channel counts / widths / rates would be converted by pydub
    (set_frame_rate, :132); that conversion is not built here and raises."""
    with wave.open(path, 'rb') as f:
        nch, width, rate, n = f.getparams()[:4]
        data = f.readframes(n)
    if nch != 1 or width != 2:
        raise ValueError(f'{path}: {nch} channel(s) x {8 * width} bit; standardize_audio is built for '
                         'mono 16-bit recordings (pydub conversion not built)')
    return rate, np.frombuffer(data, dtype='<i2').astype(np.int16)


def _write_pcm16(path, pcm, rate=16000):
    with wave.open(path, 'wb') as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(rate)
        f.writeframes(np.ascontiguousarray(pcm, dtype='<i2').tobytes())


def dbfs(pcm):
    """pydub ``AudioSegment.dBFS`` of 16-bit audio: 20 log10(audioop.rms / 2^15), audioop.rms being
    the integer part of sqrt(mean(x^2)); -inf for silence."""
    x = np.asarray(pcm, dtype=np.int64)
    if x.size == 0:
        return -float('inf')
    rms = int(np.sqrt(float(np.sum(x * x)) / x.size))
    return 20.0 * np.log10(rms / 32768.0) if rms else -float('inf')


def apply_gain(pcm, db):
    """pydub ``apply_gain``: audioop.mul(data, 2, 10 ** (db / 20)) -- per sample x * factor in
    double, clamped to [-32768, 32767] (below -32767 -> -32768), rounded towards minus infinity."""
    v = np.asarray(pcm, dtype=np.float64) * (10.0 ** (float(db) / 20.0))
    v = np.where(v > 32767.0, 32767.0, np.where(v < -32767.0, -32768.0, v))
    return np.floor(v).astype(np.int16)


def standardize_audio(source_path, target_path=None, format=None, dbfs_target=None, channels=1,
                      sampwidth=2, sample_rate=16000, noise_reduced=0, silence_remove=False,
                      noise_path=None, ctx=None, dbfs=None):
    """overlap_detection_post_processing.py:101-148 -> the standardised int16 PCM (also written to
    ``target_path``).

    What survives of the reference's steps: its first librosa.load / peak normalisation / sf.write
    of ``target_path`` (:103-114) is overwritten by the pydub export of the ORIGINAL source (:116-123),
    so it changes nothing and is not repeated.  pydub: ``set_frame_rate(16000)`` (a no-op for the
    16 kHz recordings; other rates raise), ``if dbfs:`` gain to ``dbfs`` dBFS -- note the reference
    calls it with ``dbfs=0``, which is falsy, so no gain is applied there either.  Then
    ``noise_reduced`` passes of load (x / 32768) -> the stationary noise gate against the ambient
    noise file (mmla_audio_amd.noisereduce, nr.hip) -> ``sf.write`` PCM_16 (mmla_pcm16), and the
    optional silence removal (vad_collector on the context's detector, :138-148)."""
    from . import _lib, noisereduce as nr
    from .overlap_features_generator import _load
    target = dbfs if dbfs is not None else dbfs_target
    ctx = ctx or _lib.default_context()
    if not target_path:
        target_path = source_path[:-4] + '.wav'
    rate, pcm = _read_pcm16(source_path)
    if sample_rate and rate != sample_rate:
        raise ValueError(f'{source_path}: {rate} Hz; resampling to {sample_rate} Hz is not built')
    if target:
        pcm = apply_gain(pcm, target - dbfs(pcm))
    _write_pcm16(target_path, pcm, sample_rate)
    if noise_reduced > 0:
        _, noise = _load(noise_path)
        noise = noise.astype(np.float32) / np.float32(32768.0) if noise.dtype == np.int16 else noise
        while noise_reduced > 0:
            noise_reduced -= 1
            y = pcm.astype(np.float32) / np.float32(32768.0)            # librosa.load(sr=None)
            out = nr.reduce_noise(y_noise=noise, y=y, sr=sample_rate, stationary=True)
            pcm = ctx.pcm16(out)                                           # sf.write PCM_16
            _write_pcm16(target_path, pcm, sample_rate)
    if silence_remove:
        if getattr(ctx, 'vad_streams', None) != 1:                         # the module-level Vad(3)
            ctx.vad_reset(1, 3)
        voiced, _ = ctx.vad_remove_silence([pcm], items_per_stream=1)
        pcm = voiced[0]
        _write_pcm16(target_path, pcm, sample_rate)
    return pcm


def _segment_index(name):
    """segment j of ``<base>_<j>_<rate>_split.wav``"""
    return int(name.split('_')[-3])


def post_anlysing(root_dir, model, ctx=None, noise_path=None, start_time=None):
    """overlap_detection_post_processing.py:151-226 under ``root_dir`` (the reference's Root_Dir).

    Conversations are found with os.walk over experiment/recordings/post-time/whole; ``zoom*`` files
    are standardised without, ``audio*`` files with three noise-gate passes (:182-190; the reference
    tests ``onewav.split('\\')[-1]``, a Windows separator -- this takes the base name), others are
    not standardised (the reference then fails listing their segment directory; so does this).
    Every standardised file is cut into 1.5 s segments (:194-195); per conversation ALL segment
    windows run through ONE fused OD pipeline call and the log lists the segments in os.listdir
    order of the segment directory, timestamps 1.5 s apart from the time the conversation starts.
    Returns {conversation file name: list of (segment file, label)}."""
    from . import _lib
    ctx = ctx or getattr(model, 'ctx', None) or _lib.default_context()
    noise_path = noise_path or os.path.join(root_dir, 'experiment/Ambient_Noise.wav')
    post = os.path.join(root_dir, 'experiment/recordings/post-time')
    conv, std, logs, segs, feats = [], [], [], [], []
    for (dirpath, dirnames, filenames) in os.walk(os.path.join(post, 'whole')):
        for filename in filenames:
            conv.append(os.sep.join([dirpath, filename]))
            std.append(os.path.join(post, 'standardized', filename)[:-4] + '.wav')
            logs.append(root_dir + '/experiment/logs/' + filename[:-4] + '.txt')
            segs.append(os.path.join(post, 'segments', filename)[:-4])
            feats.append(root_dir + '/experiment/recordings/post-time/features/' + filename[:-4] + '/')
    for d in feats:
        if not os.path.exists(d):
            os.mkdir(d)
    for i, onewav in enumerate(conv):
        base = os.path.basename(onewav)
        if base.startswith('zoom'):
            standardize_audio(onewav, std[i], dbfs=0, noise_reduced=0, noise_path=noise_path, ctx=ctx)
        elif base.startswith('audio'):
            standardize_audio(onewav, std[i], dbfs=0, noise_reduced=3, noise_path=noise_path, ctx=ctx)
    segmentation(os.path.join(post, 'standardized'), os.path.join(post, 'segments'), 1.5, 1.5)
    out = {}
    for i, seg_dir in enumerate(segs):
        listing = os.listdir(seg_dir)
        time = start_time if start_time is not None else datetime.today()
        rate, pcm = _read_pcm16(std[i])
        _, argmax, labels = predict_segments(pcm, model, rate, 1.5, 1.5)
        rows = []
        with open(logs[i], 'w') as f:
            f.write('segment' + '\t' + 'overlapped degree' + '\t' + 'timestamp')
            f.write('\n')
            for count, name in enumerate(listing):
                if count > 0:
                    time = time + timedelta(seconds=1.5)
                label = labels[_segment_index(name)]
                f.write(str(count) + '\t' + str(label) + '\t' + str(time))
                f.write('\n')
                rows.append((name, label))
        out[os.path.basename(conv[i])] = rows
    return out
