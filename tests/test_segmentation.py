"""Offline OD segmentation against the reference's own output.

tests/golden/seg_golden.npz was produced by running overlap_detection_post_processing.py:23-85 (the
reference source) on the synthetic WAVs regenerated here (tests/golden/make_golden.py): segment
count, file names and the SHA-256 of every segment file must match.
"""
import hashlib
import os
import wave
from datetime import datetime

import numpy as np
import pytest

from mmla_audio_amd import overlap_detection_post_processing as odpp
from oracle import synth

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'seg_golden.npz')


def _case(g, i):
    ch, n, win, step = g[f'params_{i}']
    ch, n = int(ch), int(n)
    pcm = np.stack([synth.clip(30 + i * 2 + c, n) for c in range(ch)], axis=1)
    return pcm, ch, float(win), float(step)


@pytest.mark.parametrize('i', range(4))
def test_segmentation_matches_reference(tmp_path, i):
    g = np.load(GOLD)
    pcm, ch, win, step = _case(g, i)
    src, dst = tmp_path / 'src', tmp_path / 'dst'
    src.mkdir()
    dst.mkdir()
    with wave.open(str(src / f'conv{i}.wav'), 'wb') as w:
        w.setnchannels(ch)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(pcm.astype('<i2').tobytes())
    odpp.segmentation(str(src), str(dst), win, step)
    files = sorted(os.listdir(dst / f'conv{i}'), key=lambda f: int(f.split('_')[-3]))
    assert files == list(g[f'files_{i}'])
    for j, f in enumerate(files):
        b = (dst / f'conv{i}' / f).read_bytes()
        assert len(b) == int(g[f'len_{i}_{j}'])
        assert np.array_equal(np.frombuffer(b[:44], np.uint8), g[f'head_{i}_{j}'])
        assert hashlib.sha256(b).hexdigest() == g[f'sha256_{i}'][j]


def test_segment_bounds_edge_cases():
    assert odpp.segment_bounds(84800, 16000, 1.5, 1.5) == (24000, 24000, 3)
    assert odpp.segment_bounds(64000, 16000, 1.5, 0.5) == (24000, 8000, 6)
    assert odpp.segment_bounds(23999, 16000, 1.5, 1.5)[2] == 0      # shorter than one window
    assert odpp.segment_bounds(0, 16000, 1.5, 1.5)[2] == 0


def test_write_log_format(tmp_path):
    t0 = datetime(2021, 5, 4, 12, 0, 0)
    p = tmp_path / 'log.txt'
    odpp.write_log(str(p), [0, 1, 1], start_time=t0)
    lines = p.read_text().splitlines()
    assert lines == ['segment\toverlapped degree\ttimestamp',
                     '0\tnon-overlapped\t2021-05-04 12:00:00',
                     '1\toverlapped\t2021-05-04 12:00:01.500000',
                     '2\toverlapped\t2021-05-04 12:00:03']
