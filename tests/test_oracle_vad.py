"""CPU: the VAD silence-removal restatement (oracle/vad.py) against the reference's own
frame_generator / vad_collector / rewrite run with a stub is_speech (tests/golden/vad_golden.npz),
and self-consistency of the webrtcvad restatement (oracle/webrtc_vad.py; parity unpinned: the
library is absent from this image)."""
import os

import numpy as np
import pytest

from oracle import vad, webrtc_vad

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'vad_golden.npz')


@pytest.fixture(scope='module')
def g():
    return np.load(GOLDEN)


def test_collector_matches_reference(g):
    for i, name in enumerate(g['names']):
        pcm, flags = g[f'pcm_{i}'], g[f'flags_{i}']
        fr = vad.frames(pcm)
        assert len(fr) == len(flags), name
        it = iter(flags)
        out, f2 = vad.remove_silence(pcm, lambda b, sr: next(it))
        assert np.array_equal(f2, flags), name
        assert np.array_equal(out, g[f'out_{i}']), name


def test_frame_generator_drops_exact_tail():
    assert len(vad.frames(np.zeros(4800, np.int16))) == 9     # 10 * 480 is not < 4800
    assert len(vad.frames(np.zeros(4801, np.int16))) == 10
    assert len(vad.frames(np.zeros(480, np.int16))) == 0


def test_keep_mask_trigger_rules():
    assert not vad.keep_mask([True] * 9).any()                # needs > 9 of 10 voiced
    k = vad.keep_mask([True] * 10 + [False] * 10 + [True] * 3)
    assert k[:20].all() and not k[20:].any()                  # the 10 unvoiced frames are kept too


def _tone(n, f=440.0, a=8000.0, sr=16000):
    t = np.arange(n) / sr
    return (a * np.sin(2 * np.pi * f * t)).astype(np.int16)


def test_webrtc_vad_silence_and_tone():
    v = webrtc_vad.Vad(3)
    z = np.zeros(480, np.int16)
    assert not any(v.is_speech(z.tobytes(), 16000) for _ in range(20))
    rng = np.random.default_rng(1)
    speechy = [(_tone(480, f) + rng.normal(0, 200, 480)).astype(np.int16) for f in (220, 330, 440)]
    res = [v.is_speech(s.tobytes(), 16000) for s in speechy * 5]
    assert sum(res) >= 10


def test_webrtc_vad_state_carries_across_calls():
    a, b = webrtc_vad.Vad(3), webrtc_vad.Vad(3)
    rng = np.random.default_rng(2)
    frames = [rng.normal(0, 3000, 480).astype(np.int16).tobytes() for _ in range(30)]
    ra = [a.is_speech(f, 16000) for f in frames]
    rb = [b.is_speech(f, 16000) for f in frames[:15]] + [b.is_speech(f, 16000) for f in frames[15:]]
    assert ra == rb                                  # one object, one sequence: the same answers
    assert a.frame_counter == 30 and a.noise_means != list(webrtc_vad.NOISE_MEANS)


def test_webrtc_vad_modes_ordered():
    rng = np.random.default_rng(3)
    frames = [(rng.normal(0, 1, 480) * rng.uniform(20, 4000)).astype(np.int16).tobytes() for _ in range(60)]
    counts = []
    for mode in range(4):
        v = webrtc_vad.Vad(mode)
        counts.append(sum(v.is_speech(f, 16000) for f in frames))
    assert counts[0] >= counts[3]                     # aggressiveness 3 flags the least speech
