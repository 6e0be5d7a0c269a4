"""Drop-in for the silence removal of the reference's real-time and offline loops (SURVEY.md 8f
row 2): ``webrtcvad.Vad``, ``frame_generator``, ``vad_collector`` and ``save_wave_file``
(``OverlapDetection/scripts/record_on_pc.py:33,188-295``; the SpeakerIdentification copies), with
the detector and the collector running in the ``vad`` HIP kernels (mmla_vad_* in include/mmla.h).

    from mmla_audio_amd import vad as _v
    vad = _v.Vad(3)                                     # webrtcvad.Vad(3)
    segments = _v.vad_collector(16000, 30, 300, vad, frames)

``Vad`` is one detector whose state carries across calls, like the reference's module-level
``vad``; ``remove_silence_batch`` runs many independent streams at once (one detector each).
"""
import wave

import numpy as np

from . import _lib

FRAME_MS, PADDING_MS = 30, 300


class Frame:
    """record_on_pc.py:39-43"""

    def __init__(self, bytes, timestamp, duration):   # noqa: A002 (the reference's name)
        self.bytes = bytes
        self.timestamp = timestamp
        self.duration = duration


def frame_generator(frame_duration_ms, audio, sample_rate):
    """record_on_pc.py:229-243: frames of `frame_duration_ms` from PCM bytes, the last partial (or
    exactly final) frame dropped.

    Origin: the reference's function is py-webrtcvad's example.py ``frame_generator`` (MIT licence,
    John Wiseman), which the reference copied.  These lines restate it on purpose: the frame
    boundaries (and the strict ``<`` that drops an exactly final frame) decide which samples the VAD
    collector keeps, so the drop-in must frame exactly as the reference does."""
    n = int(sample_rate * (frame_duration_ms / 1000.0) * 2)
    offset = 0
    timestamp = 0.0
    duration = (float(n) / sample_rate) / 2.0
    while offset + n < len(audio):
        yield Frame(audio[offset:offset + n], timestamp, duration)
        timestamp += duration
        offset += n


class Vad:
    """webrtcvad.Vad(mode) on the GPU: one detector (stream) kept in its own libmmla context."""

    def __init__(self, mode=3, device=None):
        self.mode = int(mode)
        self.ctx = _lib.Context(device if device is not None else 0) if device is None or \
            isinstance(device, int) else device
        self.ctx.vad_reset(1, self.mode)

    def set_mode(self, mode):
        self.__init__(mode, self.ctx)

    def is_speech(self, buf, sample_rate, length=None):
        if sample_rate != 16000:
            raise ValueError('the HIP VAD implements the 16 kHz path the reference uses')
        return bool(self.is_speech_frames([buf])[0])

    def is_speech_frames(self, frames):
        """decisions for consecutive 30 ms frames of this stream (one GPU call)"""
        if not frames:
            return np.zeros(0, bool)
        pcm = np.concatenate([np.frombuffer(f, '<i2') for f in frames])
        if any(len(f) != 960 for f in frames):
            raise ValueError('the HIP VAD takes 30 ms frames (480 samples)')
        # the frames back to back plus one sample: frame_generator then yields exactly these
        padded = np.concatenate([pcm, np.zeros(1, np.int16)])
        _, flags = self.ctx.vad_remove_silence(padded[None])
        return flags[0]


def vad_collector(sample_rate, frame_duration_ms, padding_duration_ms, vad, frames):
    """record_on_pc.py:246-295: yields the voiced segments (bytes).  The decisions of all frames
    come from one GPU call when `vad` is a mmla Vad; the ring-buffer logic is the reference's."""
    import collections
    frames = list(frames)
    if isinstance(vad, Vad) and frame_duration_ms == FRAME_MS:
        decisions = vad.is_speech_frames([f.bytes for f in frames])
    else:
        decisions = [vad.is_speech(f.bytes, sample_rate) for f in frames]
    num_padding_frames = int(padding_duration_ms / frame_duration_ms)
    ring_buffer = collections.deque(maxlen=num_padding_frames)
    triggered = False
    voiced_frames = []
    for frame, is_speech in zip(frames, decisions):
        if not triggered:
            ring_buffer.append((frame, is_speech))
            if len([f for f, s in ring_buffer if s]) > 0.9 * ring_buffer.maxlen:
                triggered = True
                voiced_frames.extend(f for f, _ in ring_buffer)
                ring_buffer.clear()
        else:
            voiced_frames.append(frame)
            ring_buffer.append((frame, is_speech))
            if len([f for f, s in ring_buffer if not s]) > 0.9 * ring_buffer.maxlen:
                triggered = False
                yield b''.join(f.bytes for f in voiced_frames)
                ring_buffer.clear()
                voiced_frames = []
    if voiced_frames:
        yield b''.join(f.bytes for f in voiced_frames)


def remove_silence_batch(pcm, lens=None, items_per_stream=1, mode=3, ctx=None, reset=True):
    """Batched save_wave_file(silence_remove=True) body: int16 [n, L] (or a list) -> list of the
    voiced PCM of every item.  Consecutive groups of `items_per_stream` items share one detector
    (processed in order); `reset=False` continues the context's detectors from earlier calls."""
    ctx = ctx or _lib.default_context()
    n = len(pcm)
    if reset or getattr(ctx, 'vad_streams', None) != n // max(items_per_stream, 1):
        ctx.vad_reset(max(n // max(items_per_stream, 1), 1), mode)
    out, _ = ctx.vad_remove_silence(pcm, lens, items_per_stream)
    return out


def save_wave_file(filepath, data, noise_reduce=False, silence_remove=False, noise=None, vad=None,
                   channels=1, sampwidth=2, framerate=16000):
    """record_on_pc.py:200-226: write the recorded frames, optionally noise-gate them against the
    ambient-noise clip `noise` (float32, as librosa.load gives it; mmla nr kernels) and write the
    result as PCM_16 like sf.write, then drop the unvoiced frames with `vad` (a mmla Vad)."""
    pcm = np.frombuffer(b''.join(data), '<i2').astype(np.int16)
    if noise_reduce:
        from .noisereduce import reduce_noise
        y = reduce_noise(y=pcm.astype(np.float32) / 32768.0, sr=framerate, y_noise=noise,
                         stationary=True)
        pcm = (vad.ctx if vad is not None else _lib.default_context()).pcm16(y)
    if silence_remove:
        if vad is None:
            raise ValueError('silence_remove needs the Vad instance (the reference module-level vad)')
        pcm = np.frombuffer(b''.join(vad_collector(framerate, FRAME_MS, PADDING_MS, vad,
                                                   frame_generator(FRAME_MS, pcm.tobytes(), framerate))),
                            '<i2')
    with wave.open(filepath, 'wb') as wf:
        wf.setnchannels(channels)
        wf.setsampwidth(sampwidth)
        wf.setframerate(framerate)
        wf.writeframes(np.asarray(pcm, '<i2').tobytes())
