"""``mmla_audio_amd.tf_compat`` (the ``import tensorflow as tf`` drop-in) on the CPU: the PNG decoder
against the reference's own ``plt.imsave`` files (od_png_golden.npz) and against PIL for every colour
type / bit depth / scanline filter, ``tf.stack(...).numpy()``, ``tf.keras.models.load_model``'s
missing-weights behaviour, and that the call-site text the GPU test executes is the reference's."""
import os
import struct
import zlib

import numpy as np
import pytest

from mmla_audio_amd import tf_compat as tf

import refsites

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, 'tests', 'golden')
REFERENCE = '/root/reference'


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason='reference checkout absent')
@pytest.mark.parametrize('site', refsites.ALL, ids=lambda s: f'{os.path.basename(s[0])}:{s[1]}')
def test_call_site_text_matches_reference(site):
    path, line, text = site
    lines = open(os.path.join(REFERENCE, path)).read().split('\n')
    want = text.rstrip('\n').split('\n')
    got = lines[line - 1:line - 1 + len(want)]
    assert [g.strip() for g in got] == [w.strip() for w in want]


def test_decode_png_of_reference_files(od_golden):
    """the PNGs the reference's generate_zcr_image -> plt.imsave wrote decode, as 3 channels, to the
    pixels make_golden.py read back with PIL (od_golden png_i)"""
    g = np.load(os.path.join(GOLDEN, 'od_png_golden.npz'))
    for i, _ in enumerate(g['names']):
        img = tf.image.decode_png(g[f'bytes_{i}'].tobytes(), 3)
        assert img.dtype == np.uint8 and img.shape == (128, 151, 3)
        assert np.array_equal(img.numpy(), od_golden[f'png_{i}'])
        rgba = tf.image.decode_png(g[f'bytes_{i}'].tobytes())
        assert rgba.shape == (128, 151, 4) and (rgba.numpy()[..., 3] == 255).all()


def test_read_file_stack_numpy(tmp_path, od_golden):
    """the record_on_pc.py:156-158 statements up to predict: [1,128,151,3] float32 in [0,255]"""
    g = np.load(os.path.join(GOLDEN, 'od_png_golden.npz'))
    p = tmp_path / 'n.png'
    p.write_bytes(g['bytes_0'].tobytes())
    image = tf.io.read_file(str(p))
    assert image.numpy() == g['bytes_0'].tobytes() and image.shape == ()
    features_data = [tf.image.decode_png(image, 3)]
    _input = tf.stack(features_data, axis=0).numpy().astype('float32')
    assert _input.shape == (1, 128, 151, 3) and _input.dtype == np.float32
    assert np.array_equal(_input[0], od_golden['png_0'].astype(np.float32))


def _png(px, ctype, depth=8, filters=None, plte=None, trns=None):
    """minimal PNG encoder with chosen scanline filters (0-4 per row)"""
    h, w = px.shape[:2]
    nc = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    if depth < 8:
        bits = np.unpackbits(px.reshape(h, w, 1).astype(np.uint8), axis=2)[:, :, 8 - depth:]
        rows = np.packbits(bits.reshape(h, -1), axis=1)
    else:
        rows = px.reshape(h, w * nc).astype(np.uint8)
    bpp = max(1, nc * depth // 8)
    raw = bytearray()
    prev = np.zeros(rows.shape[1], np.int32)
    for r in range(h):
        f = 0 if filters is None else filters[r % len(filters)]
        cur = rows[r].astype(np.int32)
        a = np.concatenate([np.zeros(bpp, np.int32), cur[:-bpp]])
        c = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]])
        b = prev
        if f == 0:
            pred = np.zeros_like(cur)
        elif f == 1:
            pred = a
        elif f == 2:
            pred = b
        elif f == 3:
            pred = (a + b) >> 1
        else:
            p = a + b - c
            pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
            pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))
        raw.append(f)
        raw += ((cur - pred) & 255).astype(np.uint8).tobytes()
        prev = cur

    def chunk(tag, data):
        return struct.pack('>I', len(data)) + tag + data + struct.pack('>I', zlib.crc32(tag + data) & 0xFFFFFFFF)
    out = b'\x89PNG\r\n\x1a\n' + chunk(b'IHDR', struct.pack('>IIBBBBB', w, h, depth, ctype, 0, 0, 0))
    if plte is not None:
        out += chunk(b'PLTE', plte.astype(np.uint8).tobytes())
    if trns is not None:
        out += chunk(b'tRNS', bytes(trns))
    # split IDAT in two to exercise concatenation
    z = zlib.compress(bytes(raw), 9)
    return out + chunk(b'IDAT', z[:len(z) // 2]) + chunk(b'IDAT', z[len(z) // 2:]) + chunk(b'IEND', b'')


@pytest.mark.parametrize('ctype', [0, 2, 4, 6])
def test_every_filter_and_colour_type(ctype):
    from PIL import Image
    import io
    rng = np.random.default_rng(ctype)
    nc = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    px = rng.integers(0, 256, (37, 29, nc), dtype=np.uint8)
    px[5:9] = px[4]                                   # runs, so Up / Paeth see equal neighbours
    data = _png(px, ctype, filters=[0, 1, 2, 3, 4, 4, 3, 1])
    got0 = tf.image.decode_png(data).numpy()
    assert np.array_equal(got0, px.reshape(got0.shape))
    pil = Image.open(io.BytesIO(data))
    for ch, mode in ((3, 'RGB'), (4, 'RGBA')):
        want = np.asarray(pil.convert(mode))
        assert np.array_equal(tf.image.decode_png(data, ch).numpy(), want), (ctype, ch)


@pytest.mark.parametrize('depth', [1, 2, 4, 8])
def test_palette_and_grey_depths(depth):
    from PIL import Image
    import io
    rng = np.random.default_rng(depth)
    n = 1 << depth
    idx = rng.integers(0, n, (11, 13), dtype=np.uint8)
    plte = rng.integers(0, 256, (n, 3), dtype=np.uint8)
    trns = rng.integers(0, 256, n // 2 + 1, dtype=np.uint8).tolist()
    data = _png(idx, 3, depth, filters=[0, 1, 2, 3, 4], plte=plte, trns=trns)
    assert np.array_equal(tf.image.decode_png(data, 3).numpy(), plte[idx])
    assert np.array_equal(tf.image.decode_png(data, 4).numpy(),
                          np.asarray(Image.open(io.BytesIO(data)).convert('RGBA')))
    grey = _png(idx, 0, depth, filters=[4, 3, 2, 1, 0])
    want = np.asarray(Image.open(io.BytesIO(grey)).convert('L'))
    assert np.array_equal(tf.image.decode_png(grey, 1).numpy()[..., 0], want)
    assert np.array_equal(tf.image.decode_png(grey, 3).numpy(), np.repeat(want[..., None], 3, 2))


def test_decode_png_rejects_bad_input():
    px = np.zeros((4, 4, 3), np.uint8)
    data = bytearray(_png(px, 2))
    with pytest.raises(ValueError, match='signature'):
        tf.image.decode_png(b'GIF89a' + bytes(data[6:]), 3)
    bad = bytearray(data)
    bad[20] ^= 1                                       # inside IHDR: CRC error
    with pytest.raises(ValueError, match='CRC'):
        tf.image.decode_png(bytes(bad), 3)
    with pytest.raises(NotImplementedError):
        tf.image.decode_png(_png(px, 2), 1)           # colour -> grey is not restated
    raw = bytes([7]) + bytes(12)                       # unknown filter type 7
    from mmla_audio_amd import _lib
    with pytest.raises(ValueError, match='filter'):
        _lib.png_unfilter(raw, 1, 12, 3)


def test_load_model_missing_weights_raises(tmp_path):
    d = tmp_path / 'timit2.0'
    (d / 'variables').mkdir(parents=True)
    (d / 'variables' / 'variables.index').write_bytes(
        open(os.path.join(GOLDEN, 'od_timit2.0_variables.index'), 'rb').read())
    with pytest.raises(FileNotFoundError):
        refsites.run(refsites.OD_LOAD, tf=tf, model_path=str(d))
    from mmla_audio_amd.tf_compat.keras import backend as K
    assert K.floatx() == 'float32' and K.clear_session() is None
