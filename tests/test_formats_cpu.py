"""CPU: the file formats at the drop-in boundary.

generate_zcr_image writes its PNG through write_png_rgba: with matplotlib present the bytes are
those of the reference's plt.imsave(img, origin="lower") (overlap_features_generator.py:151) for
the same pixels; without it a minimal encoder whose decoded RGB is the same.
"""
import builtins

import numpy as np
import pytest

from mmla_audio_amd.overlap_features_generator import write_png_rgba


def _img():
    rng = np.random.default_rng(3)
    img = rng.random((128, 151, 3))
    img[..., 2] = img[..., 1]          # G = B = 1 - norm in the reference
    return img


def test_png_bytes_equal_plt_imsave(tmp_path):
    plt = pytest.importorskip('matplotlib.pyplot')
    img = _img()
    plt.imsave(str(tmp_path / 'ref.png'), img, origin='lower')
    q = np.trunc(img[::-1] * 255).astype(np.uint8)       # the kernel's flipped, truncated pixels
    write_png_rgba(str(tmp_path / 'ours.png'), q)
    assert (tmp_path / 'ours.png').read_bytes() == (tmp_path / 'ref.png').read_bytes()


def test_png_fallback_encoder_decodes_to_pixels(tmp_path, monkeypatch):
    from PIL import Image
    real_import = builtins.__import__

    def no_matplotlib(name, *a, **k):
        if name.startswith('matplotlib'):
            raise ImportError(name)
        return real_import(name, *a, **k)

    monkeypatch.setattr(builtins, '__import__', no_matplotlib)
    q = np.trunc(_img() * 255).astype(np.uint8)
    write_png_rgba(str(tmp_path / 'x.png'), q)
    monkeypatch.setattr(builtins, '__import__', real_import)
    im = Image.open(tmp_path / 'x.png')
    assert im.mode == 'RGBA'
    assert np.array_equal(np.asarray(im.convert('RGB')), q)
    assert (np.asarray(im)[..., 3] == 255).all()
