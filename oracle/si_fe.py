"""SpeakerIdentification front-end oracle (numpy, float64) -- TEST INFRASTRUCTURE ONLY.

Restates ``input_feature_gen`` (``SpeakerIdentification/scripts/speaker_identification.py:372-398``):
``wav.read`` int16 -> ``len < 4000`` => 'silent' -> ``python_speech_features.mfcc(sig, rate,
winlen=0.025, winstep=0.01, nfft=512)`` -> ``delta`` twice -> concat 39 -> pad / truncate to 256.

python_speech_features is not installed in this image; ``mfcc``/``fbank``/``framesig``/``powspec``/
``get_filterbanks``/``lifter`` below restate its published 0.6 algorithm (SURVEY.md section 8a
row a13), so that part is *parity unpinned*.  ``delta`` restates the reference's own function
(``speaker_identification.py:141-151``), which ``tests/golden`` pins by running the reference.
"""
import math

import numpy as np

SR = 16000
WINLEN = 400
WINSTEP = 160
NFFT = 512
NFILT = 26
NUMCEP = 13
CEPLIFTER = 22
PREEMPH = 0.97
MAX_FRAMES = 256          # speaker_identification.py:391-395
SILENT_LEN = 4000         # speaker_identification.py:375
EPS = np.finfo(float).eps


def hz2mel(hz):
    return 2595 * np.log10(1 + hz / 700.)


def mel2hz(mel):
    return 700 * (10 ** (mel / 2595.0) - 1)


def filterbank_bins(nfilt=NFILT, nfft=NFFT, samplerate=SR, lowfreq=0, highfreq=None):
    highfreq = highfreq or samplerate / 2
    melpoints = np.linspace(hz2mel(lowfreq), hz2mel(highfreq), nfilt + 2)
    return np.floor((nfft + 1) * mel2hz(melpoints) / samplerate)


def get_filterbanks(nfilt=NFILT, nfft=NFFT, samplerate=SR, lowfreq=0, highfreq=None):
    """psf.get_filterbanks -> float64 [nfilt, nfft//2 + 1]."""
    b = filterbank_bins(nfilt, nfft, samplerate, lowfreq, highfreq)
    fbank = np.zeros([nfilt, nfft // 2 + 1])
    for j in range(nfilt):
        for i in range(int(b[j]), int(b[j + 1])):
            fbank[j, i] = (i - b[j]) / (b[j + 1] - b[j])
        for i in range(int(b[j + 1]), int(b[j + 2])):
            fbank[j, i] = (b[j + 2] - i) / (b[j + 2] - b[j + 1])
    return fbank


def preemphasis(signal, coeff=PREEMPH):
    return np.append(signal[0], signal[1:] - coeff * signal[:-1])


def num_frames(slen, frame_len=WINLEN, frame_step=WINSTEP):
    if slen <= frame_len:
        return 1
    return 1 + int(math.ceil((1.0 * slen - frame_len) / frame_step))


def framesig(sig, frame_len=WINLEN, frame_step=WINSTEP):
    """psf.sigproc.framesig with a rectangular window (winfunc default ``numpy.ones``)."""
    slen = len(sig)
    nf = num_frames(slen, frame_len, frame_step)
    padlen = int((nf - 1) * frame_step + frame_len)
    padsignal = np.concatenate((sig, np.zeros((padlen - slen,))))
    idx = np.arange(frame_len)[None, :] + frame_step * np.arange(nf)[:, None]
    return padsignal[idx] * np.ones((frame_len,))


def powspec(frames, nfft=NFFT):
    return 1.0 / nfft * np.square(np.absolute(np.fft.rfft(frames, nfft)))


def fbank(signal, samplerate=SR, nfilt=NFILT, nfft=NFFT):
    signal = preemphasis(signal, PREEMPH)
    frames = framesig(signal, WINLEN, WINSTEP)
    pspec = powspec(frames, nfft)
    energy = np.sum(pspec, 1)
    energy = np.where(energy == 0, EPS, energy)
    fb = get_filterbanks(nfilt, nfft, samplerate)
    feat = np.dot(pspec, fb.T)
    feat = np.where(feat == 0, EPS, feat)
    return feat, energy


def dct2_ortho(x):
    """scipy.fftpack.dct(x, type=2, axis=1, norm='ortho') restated as a matrix product."""
    n = x.shape[1]
    k = np.arange(n)[:, None]
    m = np.arange(n)[None, :]
    c = np.cos(np.pi * k * (2 * m + 1) / (2 * n)) * np.sqrt(2.0 / n)
    c[0] *= 1 / np.sqrt(2.0)
    return x @ c.T


def lifter(cepstra, L=CEPLIFTER):
    n = np.arange(cepstra.shape[1])
    lift = 1 + (L / 2.) * np.sin(np.pi * n / L)
    return lift * cepstra


def mfcc(signal, samplerate=SR):
    """psf.mfcc(sig, rate, winlen=0.025, winstep=0.01, nfft=512) (speaker_identification.py:386)."""
    feat, energy = fbank(np.asarray(signal), samplerate)
    feat = np.log(feat)
    try:
        import scipy.fftpack
        feat = scipy.fftpack.dct(feat, type=2, axis=1, norm='ortho')[:, :NUMCEP]
    except ImportError:   # pragma: no cover - scipy is present in this image
        feat = dct2_ortho(feat)[:, :NUMCEP]
    feat = lifter(feat, CEPLIFTER)
    feat[:, 0] = np.log(energy)
    return feat


def delta(feat, N):
    """speaker_identification.py:141-151 (edge-padded regression, denominator 2*sum(n^2))."""
    feat = np.asarray(feat)
    denominator = 2 * sum([i ** 2 for i in range(1, N + 1)])
    padded = np.pad(feat, ((N, N), (0, 0)), mode='edge')
    w = np.arange(-N, N + 1)
    out = np.empty_like(feat)
    for t in range(len(feat)):
        out[t] = np.dot(w, padded[t:t + 2 * N + 1]) / denominator
    return out


def features_39(pcm):
    """mfcc + delta + delta-delta -> float64 [T, 39] (speaker_identification.py:386-389)."""
    m = mfcc(np.asarray(pcm, dtype=np.int16), SR)
    d = delta(m, 2)
    dd = delta(d, 2)
    return np.concatenate((m, d, dd), axis=1)


def input_feature_gen(pcm):
    """speaker_identification.py:372-398 on int16 PCM -> 'silent' | float64 [1, 256, 39]."""
    pcm = np.asarray(pcm, dtype=np.int16)
    if len(pcm) < SILENT_LEN:
        return 'silent'
    f = features_39(pcm)
    if f.shape[0] < MAX_FRAMES:
        f = np.concatenate((f, np.zeros((MAX_FRAMES - f.shape[0], 39))), axis=0)
    else:
        f = f[:MAX_FRAMES, :]
    return np.asarray([f])


def conversation_chunks(pcm):
    """Whole-conversation SI features chunked into 256-frame windows
    (speaker_identification_post_processing.py:255-269) -> float64 [S, 256, 39]."""
    f = features_39(np.asarray(pcm, dtype=np.int16))
    s = math.ceil(f.shape[0] / MAX_FRAMES)
    f = np.concatenate((f, np.zeros((s * MAX_FRAMES - f.shape[0], 39))), axis=0)
    return f.reshape(s, MAX_FRAMES, 39)
