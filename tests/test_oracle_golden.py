"""CPU: the oracle against the golden vectors produced by running the reference's own source
(tests/golden/make_golden.py).  These pin the oracle's restatement of the reference glue."""
import numpy as np
import pytest

from oracle import od_fe, si_fe


def test_od_features_match_reference_glue(od_golden):
    for i, name in enumerate(od_golden['names']):
        f = od_fe.od_features(od_golden[f'pcm_{i}'])
        # generate_mels -> (s_db, s_db_norm): same float32 bits as the reference loop
        assert np.array_equal(f['db'], od_golden[f'db_{i}'], equal_nan=True), name
        assert np.array_equal(f['norm'], od_golden[f'norm_{i}'], equal_nan=True), name
        assert np.array_equal(f['zcr'], od_golden[f'zcr_{i}']), name
        # plt.imsave(origin='lower') -> PNG -> decode_png(3): the model input, bit-exact
        # (numpy-1.21 float64 '1 - x' vs numpy-2 float32: allow 1 LSB on 1e-4 of pixels)
        d = f['png_rgb'].astype(int) - od_golden[f'png_{i}'].astype(int)
        assert np.abs(d).max() <= 1 and np.count_nonzero(d) <= 1e-4 * d.size, name


def test_od_image_assembly(od_golden):
    f = od_fe.od_features(od_golden['pcm_0'])
    img = od_golden['image_0']
    assert img.shape == (128, 151, 3) and img.dtype == np.float64
    assert np.array_equal(img[..., 0], f['image'][..., 0])
    assert np.abs(img[..., 1:] - f['image'][..., 1:]).max() < 1e-7   # f32 vs f64 '1 - x'


def test_od_digital_silence_is_nan(od_golden):
    i = list(od_golden['names']).index('digital_zeros')
    assert np.isnan(od_golden[f'norm_{i}']).all()
    assert (od_golden[f'png_{i}'][..., 1:] == 0).all()


def test_si_features_match_reference_glue(si_golden):
    for i, name in enumerate(si_golden['names']):
        x = si_fe.input_feature_gen(si_golden[f'pcm_{i}'])
        if bool(si_golden[f'silent_{i}']):
            assert isinstance(x, str) and x == 'silent', name
            continue
        assert x.shape == (1, 256, 39)
        assert np.array_equal(x, si_golden[f'feat_{i}']), name


def test_delta_matches_reference(si_golden):
    assert np.array_equal(si_fe.delta(si_golden['delta_in'], 2), si_golden['delta_out'])
    assert np.array_equal(si_fe.delta(si_fe.delta(si_golden['delta_in'], 2), 2), si_golden['delta2_out'])


# ---- self-consistency known-answer tests, in place of absent library goldens ----

def test_zcr_known_answers():
    alt = np.tile(np.array([1000, -1000], np.int16), 12000)
    z = od_fe.generate_zcr(alt)[0]
    assert np.allclose(z[2:-2], 399 / 400)
    dc = np.full(24000, 500, np.int16)
    assert np.all(od_fe.generate_zcr(dc)[0] == 0)


def test_mel_basis_shape_and_sparsity():
    m = od_fe.mel_basis()
    assert m.shape == (128, 201) and m.dtype == np.float32
    nnz = (m != 0).sum(axis=1)
    assert nnz.min() >= 1 and nnz.max() <= 9 and nnz.sum() == 394
    # every row's support is a contiguous run of bins
    for r in m:
        idx = np.nonzero(r)[0]
        assert np.array_equal(idx, np.arange(idx[0], idx[-1] + 1))


def test_sine_peaks_in_right_band():
    t = np.arange(24000) / 16000
    f0 = 40 * 16000 / 400          # bin 40 centre, 1600 Hz
    pcm = (10000 * np.sin(2 * np.pi * f0 * t)).astype(np.int16)
    s = od_fe.melspectrogram(od_fe.load_int16(pcm))
    band = np.argmax(s[:, 75])
    m = od_fe.mel_basis()
    assert m[band, 40] == m[:, 40].max()


def test_psf_filterbank_bins():
    b = si_fe.filterbank_bins().astype(int).tolist()
    assert b == [0, 2, 4, 7, 10, 13, 16, 20, 24, 29, 34, 40, 46, 53, 60, 68, 77, 87, 97, 109,
                 122, 136, 152, 169, 188, 209, 231, 256]


def test_si_zero_clip_is_log_eps():
    x = si_fe.input_feature_gen(np.zeros(24000, np.int16))
    assert np.allclose(x[0, :149, 0], np.log(np.finfo(float).eps))
    assert np.all(x[0, 149:] == 0)


def test_delta_ramp():
    ramp = np.arange(20, dtype=np.float64)[:, None] * np.ones((1, 13)) * 3.0
    d = si_fe.delta(ramp, 2)
    assert np.allclose(d[2:-2], 3.0)


def test_frame_counts():
    assert si_fe.num_frames(24000) == 149
    assert si_fe.num_frames(40000) == 249
    assert si_fe.num_frames(40960) == 255
    assert si_fe.num_frames(400) == 1
    assert od_fe.N_FRAMES == 151
