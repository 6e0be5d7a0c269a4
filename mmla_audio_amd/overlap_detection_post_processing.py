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
"""
import os
import wave
from datetime import datetime, timedelta

import numpy as np

OVERLAP_DEGREE = {'0': 'non-overlapped', '1': 'overlapped'}   # overlap_detection_post_processing.py:18


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
    return probs, am, [OVERLAP_DEGREE[str(int(k))] for k in am]


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
            f.write(str(count) + '\t' + str(OVERLAP_DEGREE[str(int(k))]) + '\t' + str(time))
            f.write('\n')
