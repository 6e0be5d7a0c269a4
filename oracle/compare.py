"""Probability comparison rules for the parity tests and bench.py's parity sample -- TEST
INFRASTRUCTURE ONLY (never imported by the product path).

The reference's own check of a converted model is argmax equality over its inputs
(OverlapDetection/scripts/tfl_convert.py:73-87); its consumers read argmax and the per-class
probability (SpeakerIdentification/scripts/speaker_identification.py:401-410).  An absolute
probability bar is meaningless at p ~ 1/630, so probabilities are compared as LOG-probabilities
(a relative bound at every magnitude), and an argmax disagreement is excused only where the
reference's top-2 LOG-margin is below the comparison bar itself.
"""
import numpy as np

LOGP_TOL = 1e-4          # max |log p_gpu - log p_ref|
TIE_LOG_MARGIN = 2 * LOGP_TOL   # top-2 log-margin below which the argmax is not decided by the bar


def logp_err(p, ref):
    """max |log p - log ref| over all entries (float64 logs; an exact 0 on either side is -inf, so it
    only matches an exact 0)."""
    p = np.asarray(p, np.float64)
    ref = np.asarray(ref, np.float64)
    with np.errstate(divide='ignore'):
        a, b = np.log(p), np.log(ref)
    both = np.isneginf(a) & np.isneginf(b)
    d = np.where(both, 0.0, np.abs(a - b))
    return float(d.max()) if d.size else 0.0


def log_margin(ref):
    """top-1 minus top-2 log-probability of each row"""
    with np.errstate(divide='ignore'):
        s = np.sort(np.log(np.asarray(ref, np.float64)), axis=1)
    return s[:, -1] - s[:, -2]


def near_ties(ref):
    return log_margin(ref) < TIE_LOG_MARGIN


def argmax_report(p, ref):
    """(agree, disagree_non_tie, ties) counts"""
    a = np.asarray(p).argmax(1)
    b = np.asarray(ref).argmax(1)
    tie = near_ties(ref)
    agree = a == b
    return int(agree.sum()), int((~agree & ~tie).sum()), int(tie.sum())


def argmax_ok(p, ref):
    return argmax_report(p, ref)[1] == 0


# OD front-end bars: normalised log-mel <= 1e-4, dB <= 5e-3, exact crossing counts,
# image R exact and G/B <= 1 LSB (on <= 1e-4 of the pixel values of a test: od_lsb_budget)
OD_NORM_TOL = 1e-4
OD_DB_TOL = 5e-3


def od_clip_compare(f, i, ref, tag):
    """clip i of a GPU feature dict f (keys present of db / norm / zcr / img) against the oracle's
    od_features(...) dict; -> (pixel values 1 LSB off, pixel values) for od_lsb_budget"""
    nan = np.isnan(ref['norm'])
    if 'norm' in f:
        assert np.array_equal(np.isnan(f['norm'][i]), nan), tag
        if (~nan).any():
            err = np.abs(f['norm'][i][~nan] - ref['norm'][~nan]).max()
            assert err <= OD_NORM_TOL, f'{tag}: norm err {err}'
    if 'db' in f and (~nan).any():
        derr = np.abs(f['db'][i] - ref['db']).max()
        assert derr <= OD_DB_TOL, f'{tag}: dB err {derr}'
    if 'zcr' in f:
        counts = np.rint(f['zcr'][i] * 400).astype(int)
        assert np.array_equal(counts, np.rint(ref['zcr'][0] * 400).astype(int)), tag
        assert np.abs(f['zcr'][i] - ref['zcr'][0]).max() < 1e-7
    if 'img' not in f:
        return 0, 0
    img = f['img'][i].astype(int)
    want = ref['png_rgb'].astype(int)
    assert np.array_equal(img[..., 0], want[..., 0]), f'{tag}: R channel'
    d = np.abs(img - want)
    assert d.max() <= 1, f'{tag}: {d.max()} LSB'
    return np.count_nonzero(d), d.size


def od_lsb_budget(counts):
    """<= 1 LSB on <= 1e-4 of the pixel values, over all clips of a test"""
    off, tot = np.sum(np.asarray(counts, np.int64).reshape(-1, 2), axis=0)
    assert off <= 1e-4 * max(tot, 1), f'{off} of {tot} pixel values 1 LSB off'
