"""Offline SpeakerIdentification post-processing on the MI355X path.

Mirrors SpeakerIdentification/scripts/speaker_identification_post_processing.py:

* ``segmentation`` (:58-120) -- the same cutter as the OverlapDetection script (shared code in
  overlap_detection_post_processing.py, byte-identical segment WAVs).
* ``read_wave_file`` (:123-133).
* ``post_analyse_conversation(...)`` -- one conversation of ``post_analysing`` (:191-312) with the
  reference's semantics on the GPU:
    1. every 2.56 s segment, in order, through the silence removal with ONE detector
       (the module-level ``webrtcvad.Vad(3)``, :26, :225-251): segments whose voiced PCM has fewer
       than 4000 samples are 'silent';
    2. MFCC + deltas of the WHOLE conversation, zero-padded to 256-frame windows (:253-269,
       ``conversation_features`` -> si_fe kernel);
    3. ONE batched ``model.predict`` of all windows (:271-272) -> window i is labelled 'silent' when
       segment i was silent, else ``speaker_id_dict[str(argmax)]`` (:274-312);
  ``write_log`` writes the reference's TSV (a header before window 0, timestamps advancing 2.56 s
  before every line).
* ``speaker_id_dict_from_corpus(files)`` -- :193-199 (``{str(i): file[:-4]}`` in listing order).
"""
import wave
from datetime import datetime, timedelta

import numpy as np

from . import _lib
from .overlap_detection_post_processing import segment_bounds, segmentation  # noqa: F401
from .speaker_identification import conversation_features

SILENT_LEN = 4000
SEGMENT_SECONDS = 2.56


def read_wave_file(filepath):
    """(:123-133) -> (PCM bytes, sample rate); mono 16-bit only, like the reference's asserts."""
    with wave.open(filepath, 'rb') as wf:
        assert wf.getnchannels() == 1
        assert wf.getsampwidth() == 2
        sample_rate = wf.getframerate()
        assert sample_rate in (8000, 16000, 32000, 48000)
        return wf.readframes(wf.getnframes()), sample_rate


def speaker_id_dict_from_corpus(files):
    """(:193-199) labels of the registered speakers in corpus listing order"""
    return {str(i): f[:-4] for i, f in enumerate(files)}


def silent_segments(segments, ctx=None, vad_mode=3, reset=True, speech=None):
    """Indices of the segments that are silent after silence removal (:225-251), one detector over
    the segments in order.  segments: list of int16 arrays; `speech` (per-segment frame decisions)
    replaces the detector when given.  -> (indices, voiced PCM per segment)"""
    ctx = ctx or _lib.default_context()
    if not segments:
        return [], []
    if speech is not None:
        voiced = ctx.vad_collect(list(segments), speech)
    else:
        if reset or getattr(ctx, 'vad_streams', None) != 1:
            ctx.vad_reset(1, vad_mode)
        voiced, _ = ctx.vad_remove_silence(list(segments), items_per_stream=len(segments))
    return [i for i, v in enumerate(voiced) if len(v) < SILENT_LEN], voiced


def post_analyse_conversation(whole_pcm, segments, model, speaker_id_dict, ctx=None, vad_mode=3,
                              speech=None, reset_vad=False):
    """-> (labels per 256-frame window: speaker name or 'silent', probabilities [S, K], silent
    segment indices).  ``model`` is a SpeakerIdModel (models.load_model) or anything with
    ``predict([S, 256, 39])``; `speech` as in silent_segments.

    The reference keeps ONE module-level ``webrtcvad.Vad(3)`` (:26) for every conversation of
    post_analysing, so its adaptive state carries from one conversation to the next: the context's
    detector is created on the first call and kept by later ones (``reset_vad=True`` starts afresh)."""
    ctx = ctx or getattr(model, 'ctx', None) or _lib.default_context()
    silent, _ = silent_segments(segments, ctx, vad_mode, reset=reset_vad, speech=speech)
    test_x = conversation_features(np.asarray(whole_pcm, np.int16))
    results = model.predict(test_x)
    labels = []
    for i in range(results.shape[0]):
        if i in silent:
            labels.append('silent')
        else:
            labels.append(speaker_id_dict[str(int(np.argmax(results[i], axis=0)))])
    return labels, results, silent


def write_log(log_path, labels, start_time=None):
    """The TSV of post_analysing (:274-312): header before window 0, then one line per window with
    the timestamp advanced by 2.56 s first."""
    time = start_time or datetime.today()
    with open(log_path, 'a') as f:
        for i, speaker in enumerate(labels):
            time = time + timedelta(seconds=SEGMENT_SECONDS)
            if i == 0:
                f.write('segment' + '\t' + 'speaker' + '\t' + 'timestamp')
                f.write('\n')
            f.write(str(i) + '\t' + str(speaker) + '\t' + str(time))
            f.write('\n')
