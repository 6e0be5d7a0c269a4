"""Deterministic synthetic 16 kHz int16 clips generated directly in HBM (torch on the GPU).

Same five classes as SURVEY.md 8d / ``oracle/synth.py`` (voiced harmonic synth; two overlapped
talkers; white noise at -20/-40/-60 dBFS; near-silence / digital zeros; full-scale clipped), drawn
from a seeded ``torch.Generator`` so every clip has distinct bytes and a run is reproducible on a
given device.  Used by bench.py for the 65 536-clip batches (5.2 GB of PCM per GPU) that would take
minutes to synthesise on the host.
"""
import math

import torch

SR = 16000


def _voiced(g, n, L, dev):
    t = torch.arange(L, device=dev, dtype=torch.float64)[None] / SR
    u = lambda lo, hi: lo + (hi - lo) * torch.rand((n, 1), generator=g, device=dev, dtype=torch.float64)
    f0, vr, vp = u(100, 250), u(4, 7), u(0, 2 * math.pi)
    # phase = 2 pi * integral(f0 + 40 sin(2 pi vr t + vp)) dt, in closed form (float64)
    phase = 2 * math.pi * f0 * t + (40.0 / vr) * (torch.cos(vp) - torch.cos(2 * math.pi * vr * t + vp))
    x = torch.zeros((n, L), device=dev, dtype=torch.float32)
    for k in range(1, 31):
        ph = torch.remainder(k * phase + u(0, 2 * math.pi), 2 * math.pi).float()
        x += torch.sin(ph) / k
    am = 0.55 + 0.45 * torch.sin(2 * math.pi * u(2, 5) * t + u(0, 2 * math.pi)).float()
    x *= am
    return x / (x.abs().amax(dim=1, keepdim=True) + 1e-12)


def make_clips(n, clip_len=40000, seed=20261015, device='cuda', chunk=1024, start_index=0):
    """-> torch.int16 [n, clip_len] on `device`; clip i has class (start_index + i) % 5."""
    out = torch.empty((n, clip_len), dtype=torch.int16, device=device)
    g = torch.Generator(device=device)
    g.manual_seed(seed + 7919 * start_index)
    peak = 10 ** (-6 / 20)
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        cls = (torch.arange(c0, c0 + m, device=device) + start_index) % 5
        a = _voiced(g, m, clip_len, device)
        b = _voiced(g, m, clip_len, device)
        noise = torch.randn((m, clip_len), generator=g, device=device)
        lvl = torch.tensor([10 ** (-20 / 20), 10 ** (-40 / 20), 10 ** (-60 / 20)], device=device)
        lvl = lvl[torch.randint(0, 3, (m,), generator=g, device=device)][:, None]
        x = torch.zeros((m, clip_len), device=device)
        c = cls[:, None]
        x = torch.where(c == 0, peak * a + 0.01 * peak * noise, x)
        ab = a + b
        ab = peak * ab / (ab.abs().amax(dim=1, keepdim=True) + 1e-12) + 0.01 * peak * noise
        x = torch.where(c == 1, ab, x)
        x = torch.where(c == 2, lvl * noise / 3.0, x)
        lsb = torch.randint(-1, 2, (m, clip_len), generator=g, device=device).float() / 32767.0
        zeros = (torch.rand((m, 1), generator=g, device=device) < 0.5).float()
        x = torch.where(c == 3, lsb * (1 - zeros), x)
        x = torch.where(c == 4, 4.0 * a, x)
        out[c0:c0 + m] = torch.clamp(torch.round(x * 32767.0), -32768, 32767).to(torch.int16)
    return out
