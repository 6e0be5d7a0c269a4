"""``tf.image.decode_png`` for ``record_on_pc.py:157`` / ``overlap_detection_post_processing.py:205``.

PNG container parsing, CRC checks and the channel conversions run here; inflate is zlib's (the
library libpng uses) and the scanline reconstruction is native (``mmla_png_unfilter``).  Decodes
non-interlaced 1/2/4/8-bit images of every colour type, which covers what ``plt.imsave`` writes
(8-bit RGBA, ``generate_zcr_image``).  ``channels=3`` drops an alpha channel without compositing
and expands grey / palette images, as TF's decoder does.  What TF would do with a 16-bit or Adam7
image, or a colour-to-grey conversion, is not restated: those raise instead of guessing.
"""
import struct
import zlib

import numpy as np

_SIG = b'\x89PNG\r\n\x1a\n'
_NCHAN = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}      # PNG colour type -> samples per pixel


def _chunks(data):
    if data[:8] != _SIG:
        raise ValueError('decode_png: not a PNG file (bad signature)')
    p = 8
    while p + 12 <= len(data):
        n, tag = struct.unpack('>I4s', data[p:p + 8])
        body = data[p + 8:p + 8 + n]
        if len(body) != n or p + 12 + n > len(data):
            raise ValueError(f'decode_png: truncated {tag!r} chunk')
        crc, = struct.unpack('>I', data[p + 8 + n:p + 12 + n])
        if zlib.crc32(tag + body) & 0xFFFFFFFF != crc:
            raise ValueError(f'decode_png: CRC error in the {tag.decode("latin-1")} chunk')
        yield tag, body
        if tag == b'IEND':
            return
        p += 12 + n
    raise ValueError('decode_png: missing IEND chunk')


def _decode_native(data):
    """-> (uint8 [h, w, c] with c = the file's samples per pixel after palette expansion,
    alpha present)"""
    from .. import _lib
    ihdr, plte, trns, idat = None, None, None, []
    for tag, body in _chunks(data):
        if tag == b'IHDR':
            ihdr = struct.unpack('>IIBBBBB', body)
        elif tag == b'PLTE':
            plte = np.frombuffer(body, np.uint8).reshape(-1, 3)
        elif tag == b'tRNS':
            trns = body
        elif tag == b'IDAT':
            idat.append(body)
    if ihdr is None or not idat:
        raise ValueError('decode_png: missing IHDR or IDAT')
    w, h, depth, ctype, comp, filt, interlace = ihdr
    if ctype not in _NCHAN or comp != 0 or filt != 0:
        raise ValueError(f'decode_png: invalid IHDR (colour type {ctype})')
    if interlace:
        raise NotImplementedError('decode_png: Adam7-interlaced PNGs are not supported')
    if depth == 16:
        raise NotImplementedError('decode_png: 16-bit PNGs are not supported (TF\'s 16 -> 8-bit '
                                  'reduction is not restated)')
    if depth not in (1, 2, 4, 8) or (depth != 8 and ctype not in (0, 3)):
        raise ValueError(f'decode_png: invalid bit depth {depth} for colour type {ctype}')
    nc = _NCHAN[ctype]
    row_bytes = (w * nc * depth + 7) // 8
    raw = zlib.decompress(b''.join(idat))
    rows = _lib.png_unfilter(raw[:h * (row_bytes + 1)], h, row_bytes, max(1, nc * depth // 8))
    if depth == 8:
        px = rows.reshape(h, w, nc)
    else:
        bits = np.unpackbits(rows, axis=1)[:, :w * depth].reshape(h, w, depth)
        px = (bits * (1 << np.arange(depth - 1, -1, -1, dtype=np.uint8))).sum(2, dtype=np.uint16)
        px = px.astype(np.uint8)[..., None]
        if ctype == 0:                                  # libpng expand_gray_1_2_4_to_8
            px = px * np.uint8(255 // ((1 << depth) - 1))
    if ctype == 3:
        if plte is None:
            raise ValueError('decode_png: palette image without PLTE')
        idx = px[..., 0]
        if idx.max(initial=0) >= len(plte):
            raise ValueError('decode_png: palette index out of range')
        rgb = plte[idx]
        if trns is None:
            return rgb
        alpha = np.full(256, 255, np.uint8)
        alpha[:len(trns)] = np.frombuffer(trns, np.uint8)[:256]
        return np.concatenate([rgb, alpha[idx][..., None]], axis=2)
    return px


def decode_png(contents, channels=0, dtype=np.uint8, name=None):
    """``tf.image.decode_png(contents, channels)`` -> uint8 [h, w, channels] tensor."""
    from . import Tensor, _value
    data = _value(contents)
    if not isinstance(data, (bytes, bytearray, memoryview)):
        raise TypeError('decode_png expects the bytes of a PNG file (tf.io.read_file)')
    px = _decode_native(bytes(data))
    have = px.shape[2]
    color = have >= 3
    alpha = have in (2, 4)
    if channels == 0:
        out = px
    elif channels in (3, 4):
        rgb = px[..., :3] if color else np.repeat(px[..., :1], 3, axis=2)
        if channels == 3:
            out = rgb
        else:
            a = px[..., -1:] if alpha else np.full(px.shape[:2] + (1,), 255, np.uint8)
            out = np.concatenate([rgb, a], axis=2)
    elif channels in (1, 2):
        if color:
            raise NotImplementedError('decode_png: colour -> grey conversion is not supported')
        out = px[..., :1] if channels == 1 else (
            px if alpha else np.concatenate([px, np.full_like(px, 255)], axis=2))
    else:
        raise ValueError(f'decode_png: channels must be 0, 1, 2, 3 or 4, got {channels}')
    out = np.ascontiguousarray(out)
    dt = np.dtype(dtype)
    if dt == np.uint16:
        out = out.astype(np.uint16) * np.uint16(257)
    elif dt != np.uint8:
        raise ValueError(f'decode_png: dtype must be uint8 or uint16, got {dt}')
    return Tensor(out)
