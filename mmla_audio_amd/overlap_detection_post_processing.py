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

from .audio_segment import AudioSegment, _read_wav, load, mul

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


def segmentation(src_dir, dst_dir, win_time_stride, step_time, fixed_format=None):
    """Cut the WAVs of ``src_dir`` into ``win_time_stride``-second windows every ``step_time``
    seconds, written under ``dst_dir/<name>/`` (overlap_detection_post_processing.py:23-85).
    ``fixed_format`` = (channels, sample width, rate): the SpeakerIdentification script's variant
    (speaker_identification_post_processing.py:58-120), which sizes the windows from its 16 kHz
    module constant and writes every segment with its module's mono / 16-bit / 16 kHz header."""
    files = [os.path.join(src_dir, f) for f in os.listdir(src_dir) if f.endswith('.wav')]
    for filename in files:
        with wave.open(filename, 'rb') as f:
            nchannels, sampwidth, framerate, nframes = f.getparams()[:4]
            str_data = f.readframes(nframes)
        wave_data = np.frombuffer(str_data, dtype=np.short)
        temp_data = wave_data.reshape(-1, 2) if nchannels > 1 else wave_data   # frames x channels
        out_ch, out_width, out_rate = fixed_format or (nchannels, sampwidth, framerate)

        win_num_frames, step_num_frames, cut_num = segment_bounds(nframes, out_rate,
                                                                  win_time_stride, step_time)
        print("window frames: ", win_num_frames, "step frames: ", step_num_frames)
        step_total_num_frames = 0
        base = os.path.splitext(os.path.split(filename)[-1])[0]
        file_save_path = os.path.join(dst_dir, base)
        for j in range(cut_num):
            if not os.path.exists(file_save_path):
                os.makedirs(file_save_path)
            out_file = os.path.join(file_save_path, base + '_%d_%s_split.wav' % (j, out_rate))
            start = step_num_frames * j
            seg = np.ascontiguousarray(temp_data[start:start + win_num_frames]).astype(np.short)
            step_total_num_frames = (j + 1) * step_num_frames
            with wave.open(out_file, 'wb') as f:
                f.setnchannels(out_ch)
                f.setsampwidth(out_width)
                f.setframerate(out_rate)
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
    """(rate, int16 PCM) of a mono 16-bit WAV"""
    rate, nch, width, x = _read_wav(path)
    if nch != 1 or width != 2:
        raise ValueError(f'{path}: {nch} channel(s) x {8 * width} bit; expected mono 16-bit')
    return rate, x


def _write_pcm16(path, pcm, rate=16000, channels=1):
    with wave.open(path, 'wb') as f:
        f.setnchannels(channels)
        f.setsampwidth(2)
        f.setframerate(rate)
        f.writeframes(np.ascontiguousarray(pcm, dtype='<i2').tobytes())


def pcm_dbfs(pcm):
    """pydub ``AudioSegment.dBFS`` of 16-bit audio: 20 math.log(audioop.rms / 2^15, 10), audioop.rms being
    the integer part of sqrt(mean(x^2)); -inf for silence."""
    return AudioSegment(pcm, 16000).dBFS


def apply_gain(pcm, db):
    """pydub ``apply_gain``: audioop.mul(data, 2, 10 ** (db / 20)) -- per sample x * factor in
    double, clamped to [-32768, 32767] (below -32767 -> -32768), rounded towards minus infinity."""
    return mul(pcm, 10.0 ** (float(db) / 20.0))


def _vad_owner(ctx, owner, mode):
    """the reference keeps one module-level webrtcvad.Vad(3) per script (OD post :17, SI post :26,
    the record_on_pc modules); a context holds one detector: (re)create it when another script's
    detector or another mode was in use, else keep its adaptive state"""
    if getattr(ctx, 'vad_owner', None) != (owner, mode) or getattr(ctx, 'vad_streams', None) != 1:
        ctx.vad_reset(1, mode)   # clears ctx.vad_owner (any other reset clears it too)
        ctx.vad_owner = (owner, mode)


def remove_silence_file(path, ctx, owner, sample_rate=16000, channels=1, sampwidth=2, vad_mode=3,
                        speech=None):
    """the ``silence_remove`` tail of standardize_audio (:134-148 here, SI :174-188) and of SI
    post_analysing's per-segment loop (:227-244): read_wave_file (mono 16-bit asserts), 30 ms frames
    through the script's detector, vad_collector(sr, 30, 300), the voiced frames written back.
    ``speech`` (per-frame decisions) replaces the detector (tests).  -> voiced int16 PCM"""
    with wave.open(path, 'rb') as wf:
        assert wf.getnchannels() == 1
        assert wf.getsampwidth() == 2
        sr = wf.getframerate()
        assert sr in (8000, 16000, 32000, 48000)
        pcm = np.frombuffer(wf.readframes(wf.getnframes()), '<i2').astype(np.int16)
    if sr != 16000:
        raise ValueError(f'{path}: {sr} Hz; the GPU VAD frames 30 ms at 16 kHz')
    if speech is not None:
        voiced = ctx.vad_collect([pcm], [speech])
    else:
        _vad_owner(ctx, owner, vad_mode)
        voiced, _ = ctx.vad_remove_silence([pcm], items_per_stream=1)
    _write_pcm16(path, voiced[0], sample_rate, channels)
    return voiced[0]


def noise_gate_file(target_path, noise_path, passes, sample_rate, ctx):
    """``noise_reduced`` passes (:127-132; SI :167-172): librosa.load(target, sr=None) (float32,
    channel mean) -> nr.reduce_noise(y_noise=noise, stationary=True) on nr.hip -> sf.write PCM_16
    (mono) -> the next pass reads that file.  -> final int16 PCM, or None for no pass."""
    from . import noisereduce as nr
    if passes <= 0:
        return None
    noise, _ = load(noise_path, sr=None)
    pcm = None
    while passes > 0:
        passes -= 1
        y, _ = load(target_path, sr=None)
        out = nr.reduce_noise(y_noise=noise, y=y, sr=sample_rate, stationary=True)
        pcm = ctx.pcm16(out)
        _write_pcm16(target_path, pcm, sample_rate)
    return pcm


def standardize_audio(source_path, target_path=None, format=None, dbfs=None, channels=1,
                      sampwidth=2, sample_rate=16000, noise_reduced=0, silence_remove=False,
                      noise_path=None, ctx=None, speech=None):
    """overlap_detection_post_processing.py:101-148 (same positional order) -> the standardised
    int16 PCM written to ``target_path`` (interleaved frames when the source is multi-channel).

    The reference's first librosa.load / peak normalisation / sf.write of ``target_path``
    (:104-116) is overwritten by the pydub export of the ORIGINAL source (:118-125) and is not
    repeated.  pydub: the source's 16-bit frames (any channel count and rate: a 48 kHz stereo zoom
    export), ``set_frame_rate(sample_rate)`` = audioop.ratecv on the GPU (mmla_ratecv), ``if dbfs:``
    gain to ``dbfs`` dBFS (the reference passes dbfs=0, falsy: no gain), exported with the source's
    channel count.  Then ``noise_reduced`` passes of the stationary noise gate against the ambient
    noise file (each pass reads the file mono, writes mono PCM_16) and the optional silence removal
    (mono only, as the reference's read_wave_file asserts).  The noise file is read only when a pass
    runs (the reference reads it unconditionally)."""
    from . import _lib
    ctx = ctx or _lib.default_context()
    if not target_path:
        target_path = source_path[:-4] + '.wav'
    sound = AudioSegment.from_file(source_path, format, ctx=ctx)
    if sample_rate:
        sound = sound.set_frame_rate(sample_rate)
    if dbfs:
        sound = sound.apply_gain(dbfs - sound.dBFS)
    sound.export(target_path, format='wav')
    pcm = sound.data
    out = noise_gate_file(target_path, noise_path, noise_reduced, sample_rate, ctx)
    if out is not None:
        pcm = out
    if silence_remove:
        pcm = remove_silence_file(target_path, ctx, 'od_post', sample_rate, channels, sampwidth,
                                  speech=speech)
    return pcm


def predict_frames(x, nchannels, model, sr=16000, win_time_stride=1.5, step_time=1.5):
    """predict_segments of interleaved 16-bit frames: a mono signal goes through the fused int16
    pipeline; a multi-channel one as what librosa.load(segment, sr=None) gives each segment file --
    the float32 channel mean (x / 2^15 per channel) -- through the float front-end entry
    (mmla_od_features_f32) over the same strided windows, then OD-NET on the images."""
    x = np.ascontiguousarray(x, dtype=np.int16).reshape(-1)
    if nchannels == 1:
        return predict_segments(x, model, sr, win_time_stride, step_time)
    if sr != 16000:
        raise ValueError(f'the OD front-end is defined at 16 kHz (got {sr})')
    y = np.mean((x.astype(np.float32) / np.float32(32768.0)).reshape(-1, nchannels).T, axis=0)
    y = np.ascontiguousarray(y, dtype=np.float32)
    win, step, n = segment_bounds(y.size, sr, win_time_stride, step_time)
    if n == 0:
        return np.zeros((0, 2), np.float32), np.zeros(0, np.int32), []
    model._ensure_loaded()
    f = model.ctx.od_features_strided(y, n, step, win, db=False, norm=False, zcr=False, img=True)
    probs = model.ctx.od_forward(f['img'])
    am = probs.argmax(1).astype(np.int32)
    return probs, am, [LABELS[str(int(k))] for k in am]


def _segment_index(name):
    """segment j of ``<base>_<j>_<rate>_split.wav``"""
    return int(name.split('_')[-3])


def _window_images(x, nchannels, model, sr, win_time_stride, step_time):
    """the model-input images of every segment window (what generate_zcr_image writes as PNG) and
    their OD-NET probabilities"""
    x = np.ascontiguousarray(x, dtype=np.int16).reshape(-1)
    if nchannels == 1:
        sig = x
    else:
        sig = np.ascontiguousarray(np.mean((x.astype(np.float32) / np.float32(32768.0)).reshape(
            -1, nchannels).T, axis=0), dtype=np.float32)
    win, step, n = segment_bounds(sig.size, sr, win_time_stride, step_time)
    if n == 0:
        return np.zeros((0, 128, 151, 3), np.uint8), np.zeros((0, 2), np.float32)
    model._ensure_loaded()
    f = model.ctx.od_features_strided(sig, n, step, win, db=False, norm=False, zcr=False, img=True)
    return f['img'], model.ctx.od_forward(f['img'])


def post_anlysing(root_dir, model, ctx=None, noise_path=None, start_time=None, write_features=True):
    """overlap_detection_post_processing.py:151-226 under ``root_dir`` (the reference's Root_Dir).

    Conversations are found with os.walk over experiment/recordings/post-time/whole; ``zoom*`` files
    (any rate / channel count, e.g. 48 kHz stereo exports) are standardised without, ``audio*``
    files with three noise-gate passes (:182-190; the reference tests ``onewav.split('\\')[-1]``,
    a Windows separator -- this takes the base name), others are not standardised (the reference
    then fails listing their segment directory; so does this).  Every standardised file is cut into
    1.5 s segments (:194-195; stereo segments stay stereo); per conversation ALL segment windows run
    through one batched features + OD-NET pass (a stereo window as the float32 channel mean that
    librosa.load hands generate_zcr_image), the segment images are written as
    ``features/<conversation>/<count>.png`` like the reference's loop (:201-203; write_features=False
    skips them), and the log lists the segments in os.listdir order of the segment directory,
    timestamps 1.5 s apart from the time the conversation starts.  A listed segment whose index is
    beyond this run's windows (a stale file of an earlier, longer conversation of the same name) is
    predicted from its own file, as the reference predicts every listed file.
    Returns {conversation file name: list of (segment file, label)}."""
    from . import _lib
    from .overlap_features_generator import write_png_rgba
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
        rate, nch, _, pcm = _read_wav(std[i])
        images, probs = _window_images(pcm, nch, model, rate, 1.5, 1.5)
        labels = [LABELS[str(int(k))] for k in probs.argmax(1)]
        rows = []
        with open(logs[i], 'w') as f:
            f.write('segment' + '\t' + 'overlapped degree' + '\t' + 'timestamp')
            f.write('\n')
            for count, name in enumerate(listing):
                if count > 0:
                    time = time + timedelta(seconds=1.5)
                j = _segment_index(name)
                if 0 <= j < len(labels):
                    label, img = labels[j], images[j]
                else:   # not a window of this conversation: predict the file itself
                    r2, c2, _, x2 = _read_wav(os.path.join(seg_dir, name))
                    im2, p2 = _window_images(x2, c2, model, r2, len(x2) / c2 / r2, 1.5)
                    label, img = LABELS[str(int(p2.argmax(1)[0]))], im2[0]
                if write_features:
                    write_png_rgba(feats[i] + str(count) + '.png', img)
                f.write(str(count) + '\t' + str(label) + '\t' + str(time))
                f.write('\n')
                rows.append((name, label))
        out[os.path.basename(conv[i])] = rows
    return out
