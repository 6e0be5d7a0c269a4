"""VAD silence removal of the reference's save_wave_file -- TEST INFRASTRUCTURE ONLY.

Restates ``frame_generator`` and ``vad_collector`` (``OverlapDetection/scripts/record_on_pc.py:
229-295``, shared by the SpeakerIdentification scripts) and the rewrite loop of
``save_wave_file(silence_remove=True)`` (:214-226; ``speaker_identification_post_processing.py:
225-251``): 30 ms frames (only frames that end strictly before the end of the data), a 10-frame
ring buffer, TRIGGERED after > 90 % voiced frames in the ring, NOTTRIGGERED after > 90 % unvoiced
ones, and the voiced segments concatenated back into one PCM signal.  The collector logic is pinned
by tests/golden/vad_golden.npz (the reference's own functions run with a stub ``is_speech``,
tests/golden/make_golden.py); the per-frame decision comes from oracle/webrtc_vad.py.
"""
import numpy as np

FRAME_MS, PADDING_MS = 30, 300


def frames(pcm, sr=16000, frame_ms=FRAME_MS):
    """frame_generator (:229-243): [k*n, k*n + n) for every k with k*n + n < len (samples)"""
    n = int(sr * (frame_ms / 1000.0) * 2) // 2
    pcm = np.asarray(pcm, np.int16)
    k = 0
    out = []
    while (k + 1) * n < len(pcm):
        out.append(pcm[k * n:(k + 1) * n])
        k += 1
    return out


def keep_mask(flags, padding_frames=PADDING_MS // FRAME_MS):
    """vad_collector (:246-295) on per-frame is_speech flags -> which frames are written back"""
    keep = np.zeros(len(flags), bool)
    ring = []
    triggered = False
    voiced = []
    for i, s in enumerate(flags):
        if not triggered:
            ring.append((i, bool(s)))
            if len(ring) > padding_frames:
                ring.pop(0)
            if sum(1 for _, v in ring if v) > 0.9 * padding_frames:
                triggered = True
                voiced.extend(j for j, _ in ring)
                ring = []
        else:
            voiced.append(i)
            ring.append((i, bool(s)))
            if len(ring) > padding_frames:
                ring.pop(0)
            if sum(1 for _, v in ring if not v) > 0.9 * padding_frames:
                triggered = False
                keep[voiced] = True
                ring = []
                voiced = []
    if voiced:
        keep[voiced] = True
    return keep


def remove_silence(pcm, is_speech, sr=16000):
    """the rewrite of save_wave_file(silence_remove=True): -> (int16 voiced PCM, per-frame flags)"""
    fr = frames(pcm, sr)
    flags = [bool(is_speech(f.tobytes(), sr)) for f in fr]
    keep = keep_mask(flags)
    out = np.concatenate([f for f, k in zip(fr, keep) if k]) if keep.any() else np.zeros(0, np.int16)
    return out.astype(np.int16), np.array(flags, bool)
