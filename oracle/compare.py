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
