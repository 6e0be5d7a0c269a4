"""Numpy model of the OD front-end's MFMA dataflow (od_fe.hip v3) -- dev tool, not product.

Emulates, index for index, what the v3 kernel computes so that the fragment mappings and the
3xFP16 precision can be checked on the CPU against the float64 oracle (oracle/od_fe.py) before the
kernel runs:

  400-point real DFT of a Hann-windowed frame as two matrix stages (n = n1 + 16 n2, k = 25 k1 + k2)
    stage 1 (per n1, 16 GEMMs):  Y[n1][c] = sum_n2 A1[n1][c][n2] x'[160 f + n1 + 16 n2]
                                 c = 2 k2 + ri  (k2 = 0..12; rows 26..31 zero), window folded in A1
    stage 2 (per k2', 13 GEMMs): X[row] = sum_k A2[k2'][row][k] Z[k2'][k],  k = 2 n1 + ri
                                 rows = 16 bins x (re, im): bins 25 i + k2' and 25 (i - 8) + 25 - k2'
  operands split hi + lo in fp16 (x' = x / 2^12 exactly; A1 x 2^8, A2 x 2^8), three products per
  term into one f32 accumulator; P = (re^2 + im^2) 2^-38; mel, dB, normalisation as the kernel.

Usage: python tools/fe_mfma_model.py [n_clips]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
from oracle import od_fe, synth  # noqa: E402

N1, N2 = 16, 25


def split16(v):
    v = np.asarray(v, dtype=np.float32)
    hi = v.astype(np.float16)
    lo = (v - hi.astype(np.float32)).astype(np.float16)
    return hi, lo


def stage1_coeffs():
    """A1[n1][c][n2] (float64), window and DFT-25 folded, x 2^8."""
    w = od_fe.hann_periodic()
    a = np.zeros((N1, 32, 32))
    for n1 in range(N1):
        for k2 in range(13):
            for n2 in range(N2):
                th = 2 * np.pi * n2 * k2 / 25.0
                wv = w[n1 + 16 * n2]
                a[n1, 2 * k2, n2] = wv * np.cos(th) * 256.0
                a[n1, 2 * k2 + 1, n2] = -wv * np.sin(th) * 256.0 if k2 else 0.0
    return a


def stage2_bins(k2p):
    """bin of each output pair i (0..15) of GEMM k2' (-1: unused) and whether it reads conj(Y)."""
    bins, conj = [], []
    for i in range(16):
        if k2p == 0:
            bins.append(25 * i if i <= 8 else -1)
            conj.append(False)
        elif i < 8:
            bins.append(25 * i + k2p)
            conj.append(False)
        else:
            bins.append(25 * (i - 8) + 25 - k2p)
            conj.append(True)
    return bins, conj


def stage2_coeffs():
    """A2[k2'][row][k] (float64) x 2^8; row = 2 i + ri_out, k = 2 n1 + ri_in."""
    a = np.zeros((13, 32, 32))
    for k2p in range(13):
        bins, conj = stage2_bins(k2p)
        for i, b in enumerate(bins):
            if b < 0:
                continue
            for n1 in range(N1):
                th = 2 * np.pi * n1 * b / 400.0
                C, S = np.cos(th), -np.sin(th)
                if (n1 * b) % 200 == 0:
                    S = 0.0
                sg = -1.0 if conj[i] else 1.0
                # re = C a - sg S b ; im = S a + sg C b
                a[k2p, 2 * i, 2 * n1] = C * 256.0
                a[k2p, 2 * i, 2 * n1 + 1] = -sg * S * 256.0
                a[k2p, 2 * i + 1, 2 * n1] = S * 256.0
                a[k2p, 2 * i + 1, 2 * n1 + 1] = sg * C * 256.0
    return a


def mfma3(a_hi, a_lo, b_hi, b_lo, ksteps=2):
    """acc[M, N] of sum_k a[M,k] b[k,N] as three fp16 products per term, f32 accumulator, one
    rounding per 16-term instruction (lo-hi, hi-lo, hi-hi order)."""
    acc = np.zeros((a_hi.shape[0], b_hi.shape[1]), dtype=np.float32)
    for s in range(ksteps):
        ks = slice(16 * s, 16 * s + 16)
        for ah, bh in ((a_lo, b_hi), (a_hi, b_lo), (a_hi, b_hi)):
            p = ah[:, ks].astype(np.float64) @ bh[ks, :].astype(np.float64)
            acc = (acc.astype(np.float64) + p).astype(np.float32)
    return acc


def model_clip(pcm, a1, a2, mel_w):
    x = np.zeros(24000, dtype=np.int64)
    n = min(len(pcm), 24000)
    x[:n] = pcm[:n]
    xp = np.pad(x, 200, mode='reflect')                         # 24400
    xp = np.concatenate([xp, np.zeros(1024, dtype=np.int64)])   # garbage reads n2 >= 25 (times 0)
    xs = (xp.astype(np.float64) / 4096.0).astype(np.float32)
    xh, xl = split16(xs)
    a1h, a1l = split16(a1)
    a2h, a2l = split16(a2)
    P = np.zeros((201, 151), dtype=np.float32)
    f = np.arange(151)
    # stage 1: B1[n2][f] = x'[160 f + n1 + 16 n2]
    Y = np.zeros((N1, 32, 151), dtype=np.float32)
    for n1 in range(N1):
        idx = 160 * f[None, :] + n1 + 16 * np.arange(32)[:, None]
        Y[n1] = mfma3(a1h[n1], a1l[n1], xh[idx], xl[idx])
    Yh, Yl = split16(Y)
    for k2p in range(13):
        # Z[k][f], k = 2 n1 + ri <- Y[n1][2 k2' + ri][f]
        zh = np.zeros((32, 151), dtype=np.float16)
        zl = np.zeros((32, 151), dtype=np.float16)
        for n1 in range(N1):
            for ri in range(2):
                zh[2 * n1 + ri] = Yh[n1, 2 * k2p + ri]
                zl[2 * n1 + ri] = Yl[n1, 2 * k2p + ri]
        X = mfma3(a2h[k2p], a2l[k2p], zh, zl)
        bins, _ = stage2_bins(k2p)
        for i, b in enumerate(bins):
            if b < 0:
                continue
            re = X[2 * i] * np.float32(2.0 ** -19)
            im = X[2 * i + 1] * np.float32(2.0 ** -19)
            P[b] = (re * re + im * im).astype(np.float32)
    S = (mel_w.astype(np.float32) @ P).astype(np.float32)
    return S


def main():
    nclips = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    a1, a2 = stage1_coeffs(), stage2_coeffs()
    mel_w = od_fe.mel_basis()
    # exactness of the factorisation in float64 first
    rng = np.random.default_rng(0)
    xf = rng.standard_normal(400)
    w = od_fe.hann_periodic()
    ref = np.fft.rfft(xf * w)
    Y = np.einsum('acn,an->ac', a1[:, :, :N2], xf.reshape(N2, N1).T) / 256.0   # [n1][c]
    Xm = np.zeros(201, dtype=complex)
    for k2p in range(13):
        z = np.zeros(32)
        for n1 in range(N1):
            z[2 * n1:2 * n1 + 2] = Y[n1, 2 * k2p:2 * k2p + 2]
        out = a2[k2p] @ z / 256.0
        bins, _ = stage2_bins(k2p)
        for i, b in enumerate(bins):
            if b >= 0:
                Xm[b] = out[2 * i] + 1j * out[2 * i + 1]
    print('float64 factorisation max |err| / max |X|:', np.max(np.abs(Xm - ref)) / np.max(np.abs(ref)))

    errs, flips, npix, dbe = [], 0, 0, []
    for i in range(nclips):
        pcm = synth.clip(i)
        S = model_clip(pcm, a1, a2, mel_w)
        s_db = od_fe.power_to_db(S)
        norm = od_fe.normalize_matrix(s_db)
        o = od_fe.od_features(pcm)
        with np.errstate(invalid='ignore'):
            d = np.abs(norm - o['norm'])
        if np.all(np.isnan(o['norm'])):
            continue
        errs.append(np.nanmax(d))
        dbe.append(np.max(np.abs(s_db - o['db'])))
        img = od_fe.quantize_png(od_fe.zcr_image(norm, od_fe.generate_zcr(pcm)))
        flips += int(np.sum(img != o['png_rgb']))
        npix += img.size
    errs = np.array(errs)
    print(f'{len(errs)} clips: max |norm err| {errs.max():.3e} median {np.median(errs):.3e}; '
          f'max |dB err| {max(dbe):.3e}; pixel flips {flips}/{npix} = {flips / max(npix, 1):.2e}')


if __name__ == '__main__':
    main()
