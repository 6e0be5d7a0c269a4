"""Self-consistency of the stationary noise-reduction oracle (parity with the
absent noisereduce 2.0.x / librosa 0.8 is unpinned -- see oracle/noisereduce.py)."""
import numpy as np

from oracle import noisereduce as nr


def test_smoothing_filter_shape_and_sum():
    nf, nt = nr.grads(16000)
    assert (nf, nt) == (16, 3)
    f = nr.smoothing_filter(nf, nt)
    assert f.shape == (33, 7)
    assert abs(f.sum() - 1.0) < 1e-12 and (f > 0).all()
    assert np.allclose(f, f[::-1, ::-1])


def test_stft_istft_round_trip():
    y = np.random.default_rng(0).standard_normal(20000)
    S = nr.stft(y)
    assert S.dtype == np.complex128 and S.shape == (513, 1 + 20000 // 256)
    z = nr.istft(S)
    assert np.abs(z - y[:len(z)]).max() < 1e-12
    assert nr.stft(y.astype(np.float32)).dtype == np.complex64


def test_amp_to_db_clamps_to_top_db():
    x = np.array([[1.0, 1e-3, 0.0]])
    d = nr.amp_to_db(x)
    assert d[0, 0] == 0.0 and abs(d[0, 1] + 60.0) < 1e-9 and d[0, 2] == -80.0


def test_gate_attenuates_noise_keeps_tone():
    rng = np.random.default_rng(1)
    noise = (0.01 * rng.standard_normal(32000)).astype(np.float32)
    t = np.arange(24000) / 16000
    tone = (0.3 * np.sin(2 * np.pi * 440 * t)).astype(np.float32)
    y = (tone + 0.01 * rng.standard_normal(24000)).astype(np.float32)
    out = nr.reduce_noise(y, 16000, noise)
    assert out.dtype == np.float32 and out.shape == y.shape
    pure = nr.reduce_noise(noise[:24000], 16000, noise)
    assert np.sqrt(np.mean(pure ** 2)) < 0.2 * np.sqrt(np.mean(noise[:24000] ** 2))
    # the tone survives: correlation with the clean tone stays high
    c = np.dot(out, tone) / np.sqrt(np.dot(out, out) * np.dot(tone, tone))
    assert c > 0.98


def test_chunked_equals_unchunked_interior():
    rng = np.random.default_rng(2)
    noise = (0.01 * rng.standard_normal(16000)).astype(np.float32)
    y = (0.1 * rng.standard_normal(50000)).astype(np.float32)
    a = nr.reduce_noise(y, 16000, noise, chunk_size=20000, padding=6000)
    assert a.shape == y.shape and np.isfinite(a).all()
