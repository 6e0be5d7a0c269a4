"""Deterministic synthetic 16 kHz int16 clips -- TEST INFRASTRUCTURE ONLY.

Clip ``i`` is drawn from ``numpy.random.Generator(PCG64(20261015 + i))``; its class is ``i % 5``:
  0 harmonic "voiced" synth (f0 100-250 Hz, +-40 Hz vibrato, 30 harmonics at 1/k, 2-5 Hz AM,
    -6 dBFS peak, +1 % white noise)
  1 two overlapped talkers (sum of two class-0 synths, as data_augmentation.py:20-34 overlays)
  2 white noise at -20 / -40 / -60 dBFS
  3 near-silence (+-1 LSB) or digital zeros
  4 full-scale clipped voiced synth
"""
import numpy as np

SR = 16000
SEED0 = 20261015
N_CLASSES = 5


def _voiced(rng, n):
    t = np.arange(n) / SR
    f0 = rng.uniform(100, 250)
    vib_rate = rng.uniform(4, 7)
    vib = 40.0 * np.sin(2 * np.pi * vib_rate * t + rng.uniform(0, 2 * np.pi))
    phase = 2 * np.pi * np.cumsum(f0 + vib) / SR
    k = np.arange(1, 31)[:, None]
    x = np.sum(np.sin(k * phase[None, :] + rng.uniform(0, 2 * np.pi, size=(30, 1))) / k, axis=0)
    am = 0.55 + 0.45 * np.sin(2 * np.pi * rng.uniform(2, 5) * t + rng.uniform(0, 2 * np.pi))
    x = x * am
    x = x / (np.max(np.abs(x)) + 1e-12)
    return x


def clip(i, n=40000):
    """int16 [n] for clip index i."""
    rng = np.random.Generator(np.random.PCG64(SEED0 + i))
    c = i % N_CLASSES
    peak = 10 ** (-6 / 20)
    if c == 0:
        x = peak * _voiced(rng, n) + 0.01 * rng.standard_normal(n) * peak
    elif c == 1:
        a = _voiced(rng, n)
        b = _voiced(rng, n)
        x = a + b
        x = peak * x / (np.max(np.abs(x)) + 1e-12) + 0.01 * peak * rng.standard_normal(n)
    elif c == 2:
        lvl = 10 ** (rng.choice([-20, -40, -60]) / 20)
        x = lvl * rng.standard_normal(n) / 3.0
    elif c == 3:
        if rng.uniform() < 0.5:
            return np.zeros(n, dtype=np.int16)
        return rng.integers(-1, 2, size=n).astype(np.int16)
    else:
        x = 4.0 * _voiced(rng, n)
    return np.clip(np.round(x * 32767.0), -32768, 32767).astype(np.int16)


def batch(start, count, n=40000):
    return np.stack([clip(start + j, n) for j in range(count)])
