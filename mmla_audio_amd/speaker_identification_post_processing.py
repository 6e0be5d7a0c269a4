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
* ``standardize_audio(...)`` (:136-188): librosa.load at its default 22.05 kHz (resampy kaiser_best
  on the GPU; parity with resampy unpinned: the library is absent), peak normalisation, sf.write
  PCM_16, pydub ``set_frame_rate(16000)`` (audioop.ratecv on the GPU, bit-identical), optional gain,
  export, the noise-gate passes and the silence removal.
* ``post_analysing(root_dir, model)`` (:191-312): the directory-level driver -- every conversation's
  segment directory, stale log removed, segments sorted by index and rewritten in place by the
  silence removal with the script's one detector, then the conversation flow above.
* ``run_offline(root_dir, model)`` -- the script's ``__main__`` (:315-353) minus the transfer
  learning: standardise the corpus (silence removal) and the conversations, cut 2.56 s segments,
  post_analysing.
"""
import os
import wave
from datetime import datetime, timedelta

import numpy as np

from . import _lib
from .audio_segment import AudioSegment, load
from .overlap_detection_post_processing import (_vad_owner, _write_pcm16, noise_gate_file,
                                                remove_silence_file, segment_bounds, segmentation)  # noqa: F401
from .speaker_identification import conversation_features

VAD_OWNER = 'si_post'      # the module-level webrtcvad.Vad(3) of speaker_identification_post_processing.py:26
FRAMERATE, CHANNELS, SAMPWIDTH = 16000, 1, 2      # the script's module constants (:21-24)

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
        if reset:
            ctx.vad_owner = None
        _vad_owner(ctx, VAD_OWNER, vad_mode)
        voiced, _ = ctx.vad_remove_silence(list(segments), items_per_stream=len(segments))
    return [i for i, v in enumerate(voiced) if len(v) < SILENT_LEN], voiced


def post_analyse_conversation(whole_pcm, segments, model, speaker_id_dict, ctx=None, vad_mode=3,
                              speech=None, reset_vad=False):
    """-> (labels per 256-frame window: speaker name or 'silent', probabilities [S, K], silent
    segment indices).  ``model`` is a SpeakerIdModel (models.load_model) or anything with
    ``predict([S, 256, 39])``; `speech` as in silent_segments.

    The reference keeps ONE module-level ``webrtcvad.Vad(3)`` (:26) for every conversation of
    post_analysing, so its adaptive state carries from one conversation to the next: the context's
    detector is created on the first call and kept by later SI calls with the same mode; another
    script's detector (OD standardisation) or another mode on the same context starts a fresh one
    (``reset_vad=True`` always does)."""
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


# ---- the offline chain (standardize_audio, segmentation, post_analysing, __main__) -------------

def standardize_audio(source_path, target_path=None, format=None, dbfs=None, channels=1,
                      sampwidth=2, sample_rate=16000, noise_reduced=0, silence_remove=False,
                      noise_path=None, ctx=None, speech=None):
    """speaker_identification_post_processing.py:136-188 (same positional order) -> the
    standardised int16 PCM written to ``target_path``.

    1. ``librosa.load(source_path)``: float32 mono at librosa's DEFAULT 22050 Hz -- resampy's
       kaiser_best sinc resampler on the GPU (mmla_resample_sinc; resampy is absent here, so this
       step's parity is unpinned), skipped when the file is 22.05 kHz already;
    2. peak normalisation ``y * (1 / max|y|)`` with numpy 1.21 scalar rules (the reciprocal in
       float64, applied to the float32 array as float32) and ``sf.write(target, y, 22050)``: PCM_16
       (mmla_pcm16);
    3. pydub on THAT file: ``set_frame_rate(sample_rate)`` = audioop.ratecv 22050 -> 16000 on the
       GPU (bit-identical to audioop), ``if dbfs:`` gain, export;
    4. the noise-gate passes and the silence removal with this script's detector, as the OD script.
    ``speech`` (per-frame decisions) replaces the detector in the silence removal (tests)."""
    ctx = ctx or _lib.default_context()
    if not target_path:
        target_path = source_path[:-4] + '.wav'
    y, sr = load(source_path, ctx=ctx)
    max_peak = np.max(np.abs(y))
    with np.errstate(divide='ignore', invalid='ignore'):
        ratio = 1.0 / float(max_peak)                 # Python int / np.float32 scalar: float64
        y = y * np.float32(ratio)                     # float32 array * float64 scalar: float32 loop
    print('Previous peak: ', max_peak, 'Now peak: ', np.max(np.abs(y)))
    _write_pcm16(target_path, ctx.pcm16(y), sr)
    sound = AudioSegment.from_file(target_path, 'wav', ctx=ctx)
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
        pcm = remove_silence_file(target_path, ctx, VAD_OWNER, sample_rate, channels, sampwidth,
                                  speech=speech)
    return pcm


def segmentation_si(src_dir, dst_dir, win_time_stride, step_time):
    """the SI script's own cutter (:58-120): like the OD one, but the window is computed from the
    module's 16 kHz constant and every segment is written mono 16-bit 16 kHz (the standardised
    conversations it is called on are exactly that)."""
    return segmentation(src_dir, dst_dir, win_time_stride, step_time,
                        fixed_format=(CHANNELS, SAMPWIDTH, FRAMERATE))


def _segment_index(path):
    return int(os.path.basename(path).split('_')[-3])


def post_analysing(root_dir, model, ctx=None, start_time=None, speech_for=None):
    """speaker_identification_post_processing.py:191-312 under ``root_dir`` (the script's
    Root_Dir): speaker labels from the corpus listing, then per directory of
    experiment/recordings/post-time/segments: the stale log removed, the segments sorted by their
    index and each rewritten IN PLACE by the silence removal -- one detector for every segment of
    every conversation, the script's module-level Vad(3) -- 'silent' where fewer than 4000 samples
    survive, the whole standardised conversation's MFCC windows through ONE predict, the TSV log.
    ``speech_for(path)`` -> per-frame decisions for that segment file replaces the detector
    (tests).  -> {conversation: labels per window}"""
    ctx = ctx or getattr(model, 'ctx', None) or _lib.default_context()
    files = os.listdir(root_dir + '/experiment/corpus/')
    speaker_id_dict = speaker_id_dict_from_corpus(files)
    seg_root = root_dir + '/experiment/recordings/post-time/segments/'
    out = {}
    for directory_name in os.listdir(seg_root):
        seg_dir = seg_root + directory_name
        whole_wav_path = root_dir + '/experiment/recordings/post-time/standardized/' + directory_name + '.wav'
        log_path = root_dir + '/experiment/logs/' + directory_name + '.txt'
        if os.path.exists(log_path):
            os.remove(log_path)
        else:
            print('file not exist')
        paths = [seg_dir + '/' + f for f in os.listdir(seg_dir)]
        paths.sort(key=_segment_index)
        silent_index = []
        for segment_no, wav_path in enumerate(paths):
            voiced = remove_silence_file(wav_path, ctx, VAD_OWNER, FRAMERATE, CHANNELS, SAMPWIDTH,
                                         speech=speech_for(wav_path) if speech_for else None)
            if len(voiced) < SILENT_LEN:
                silent_index.append(segment_no)
        with wave.open(whole_wav_path, 'rb') as f:
            whole = np.frombuffer(f.readframes(f.getnframes()), '<i2').astype(np.int16)
        test_x = conversation_features(whole)
        results = model.predict(test_x)
        labels = ['silent' if i in silent_index else
                  speaker_id_dict[str(int(np.argmax(results[i], axis=0)))]
                  for i in range(results.shape[0])]
        write_log(log_path, labels, start_time)
        out[directory_name] = labels
    return out


def run_offline(root_dir, model, noise_path=None, ctx=None, start_time=None, speech_for=None):
    """The script's ``__main__`` (:315-353) without the transfer learning (training is out of
    scope: ``model`` is the already trained experiment model): standardise every corpus file in
    place (dbfs=0, silence removal), standardise the conversations of post-time/whole (zoom*: no
    noise gate, audio*: three passes), cut them into 2.56 s segments, post_analysing.
    ``speech_for(path)`` -> per-frame decisions for a file's silence removal replaces the detector
    (tests)."""
    ctx = ctx or getattr(model, 'ctx', None) or _lib.default_context()
    noise_path = noise_path or os.path.join(root_dir, 'experiment/Ambient_Noise.wav')
    for (dirpath, dirnames, filenames) in os.walk(root_dir + '/experiment/corpus/'):
        for filename in filenames:
            path = os.sep.join([dirpath, filename])
            standardize_audio(path, dbfs=0, noise_reduced=0, silence_remove=True, noise_path=noise_path,
                              ctx=ctx, speech=speech_for(path) if speech_for else None)
    whole = root_dir + '/experiment/recordings/post-time/whole/'
    for audio_file_name in os.listdir(whole):
        src = os.path.join(whole, audio_file_name)
        dst = os.path.join(root_dir + '/experiment/recordings/post-time/standardized/',
                           audio_file_name[:-4] + '.wav')
        if audio_file_name.startswith('zoom'):
            standardize_audio(src, dst, dbfs=0, noise_reduced=0, noise_path=noise_path, ctx=ctx)
        elif audio_file_name.startswith('audio'):
            standardize_audio(src, dst, dbfs=0, noise_reduced=3, noise_path=noise_path, ctx=ctx)
    segmentation_si(root_dir + '/experiment/recordings/post-time/standardized/',
                    root_dir + '/experiment/recordings/post-time/segments/', 2.56, 2.56)
    return post_analysing(root_dir, model, ctx, start_time, speech_for)
