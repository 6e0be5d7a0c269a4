"""TensorFlow tensor-bundle reader (``variables/variables.index`` + ``variables.data-*``).

SURVEY.md 8(f) row 1.  The reference ships its models as Keras 2.6 SavedModels
(``save_format='tf'``; ``OverlapDetection/timit/models/timit{1.0,2.0}/``,
``SpeakerIdentification/timit/model/``) whose ``saved_model.pb`` and ``variables.data-*`` are
listed in ``.MISSING_LARGE_BLOBS``; only ``variables.index`` ships.  This module parses the index
(a LevelDB SSTable whose values are ``BundleEntryProto`` messages) so that

* the synthetic weights used until the blobs are supplied have exactly the reference layout, and
* the moment a ``variables.data-00000-of-00001`` appears, the real trained weights load.

Format (TF ``tensor_bundle.cc`` / LevelDB ``table/format.cc``): 48-byte footer = metaindex handle,
index handle (varint64 offset/size each), zero padding, magic 0xdb4775248b80fb57.  Blocks hold
prefix-compressed entries ``<shared><non_shared><value_len><key delta><value>`` followed by a
restart array and a 5-byte trailer (compression type + crc).  The bundle writer uses no
compression.  BundleEntryProto: 1 dtype, 2 shape, 3 shard_id, 4 offset, 5 size, 6 crc32c.
"""
import os
import struct

import numpy as np

_MAGIC = 0xdb4775248b80fb57
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64, 10: np.bool_}


def _varint(b, p):
    r = 0
    s = 0
    while True:
        x = b[p]
        p += 1
        r |= (x & 0x7F) << s
        s += 7
        if x < 0x80:
            return r, p


def _block_entries(b):
    nrest = struct.unpack('<I', b[-4:])[0]
    end = len(b) - 4 - 4 * nrest
    p = 0
    key = b''
    while p < end:
        shared, p = _varint(b, p)
        nonshared, p = _varint(b, p)
        vlen, p = _varint(b, p)
        key = key[:shared] + b[p:p + nonshared]
        p += nonshared
        yield key, b[p:p + vlen]
        p += vlen


def _proto(b):
    p = 0
    out = {}
    while p < len(b):
        tag, p = _varint(b, p)
        f, w = tag >> 3, tag & 7
        if w == 0:
            v, p = _varint(b, p)
        elif w == 2:
            n, p = _varint(b, p)
            v = b[p:p + n]
            p += n
        elif w == 5:
            v = struct.unpack('<I', b[p:p + 4])[0]
            p += 4
        elif w == 1:
            v = struct.unpack('<Q', b[p:p + 8])[0]
            p += 8
        else:
            raise ValueError(f'unsupported wire type {w}')
        out.setdefault(f, []).append(v)
    return out


def _shape(b):
    dims = _proto(b).get(2, [])
    return tuple(_proto(d).get(1, [0])[0] for d in dims)


def read_index(index_path):
    """-> {key: dict(dtype, shape, shard, offset, size, crc32c)} for every tensor in the bundle."""
    data = open(index_path, 'rb').read()
    if len(data) < 48 or struct.unpack('<Q', data[-8:])[0] != _MAGIC:
        raise ValueError(f'{index_path}: not a TF tensor-bundle index (bad SSTable magic)')
    foot = data[-48:]
    p = 0
    _, p = _varint(foot, p)
    _, p = _varint(foot, p)
    io, p = _varint(foot, p)
    isz, p = _varint(foot, p)
    entries = {}
    for _, handle in _block_entries(data[io:io + isz]):
        off, q = _varint(handle, 0)
        sz, q = _varint(handle, q)
        if data[off + sz] != 0:
            raise ValueError('compressed bundle blocks are not supported')
        for key, val in _block_entries(data[off:off + sz]):
            if key == b'':
                continue          # BundleHeaderProto
            e = _proto(val)
            entries[key.decode()] = dict(
                dtype=e.get(1, [0])[0], shape=_shape(e[2][0]) if 2 in e else (),
                shard=e.get(3, [0])[0], offset=e.get(4, [0])[0], size=e.get(5, [0])[0],
                crc32c=e.get(6, [None])[0])
    return entries


def variable_shapes(index_path):
    """Model variables only (drops optimizer slots, metrics and the object graph):
    {canonical key: shape}.  Keys keep the bundle's own names minus '/.ATTRIBUTES/VARIABLE_VALUE'."""
    out = {}
    for k, e in read_index(index_path).items():
        if 'optimizer' in k or k.startswith('keras_api') or k.startswith('_') or 'save_counter' in k:
            continue
        out[k.replace('/.ATTRIBUTES/VARIABLE_VALUE', '')] = e['shape']
    return out


def canonical_names(shapes, bilstm_layer):
    """Map bundle names to the canonical ``layer_with_weights-k/var`` names used by
    ``mmla_audio_amd.weights``.  The Bidirectional layer's six tensors are stored in the bundle
    under ``variables/<i>`` (timit2.0) or ``trainable_variables/<i>`` (timit1.0, SI) in the order
    fwd kernel, fwd recurrent, fwd bias, bwd kernel, bwd recurrent, bwd bias."""
    mapping = {}
    loose = []
    for k in shapes:
        if k.startswith('layer_with_weights-'):
            mapping[k] = k
        elif k.startswith('variables/') or k.startswith('trainable_variables/'):
            loose.append(k)
    loose.sort(key=lambda s: int(s.rsplit('/', 1)[1]))
    if len(loose) != 6:
        raise ValueError(f'expected 6 Bidirectional LSTM tensors, found {loose}')
    p = f'layer_with_weights-{bilstm_layer}'
    for k, suffix in zip(loose, ('forward/kernel', 'forward/recurrent_kernel', 'forward/bias',
                                 'backward/kernel', 'backward/recurrent_kernel', 'backward/bias')):
        mapping[k] = f'{p}/{suffix}'
    return mapping


def load_bundle(model_dir, bilstm_layer):
    """Read trained weights from ``<model_dir>/variables/variables.{index,data-00000-of-00001}``.

    Raises FileNotFoundError when the data shard is absent (the reference's case today)."""
    index = os.path.join(model_dir, 'variables', 'variables.index')
    shard = os.path.join(model_dir, 'variables', 'variables.data-00000-of-00001')
    entries = read_index(index)
    if not os.path.exists(shard):
        raise FileNotFoundError(f'{shard} is absent (listed in the reference .MISSING_LARGE_BLOBS)')
    shapes = {k.replace('/.ATTRIBUTES/VARIABLE_VALUE', ''): e['shape'] for k, e in entries.items()}
    names = canonical_names(variable_shapes(index), bilstm_layer)
    out = {}
    with open(shard, 'rb') as f:
        for k, e in entries.items():
            short = k.replace('/.ATTRIBUTES/VARIABLE_VALUE', '')
            if short not in names:
                continue
            f.seek(e['offset'])
            raw = f.read(e['size'])
            arr = np.frombuffer(raw, dtype=_DTYPES[e['dtype']]).reshape(shapes[short])
            out[names[short]] = arr.astype(np.float32)
    return out
