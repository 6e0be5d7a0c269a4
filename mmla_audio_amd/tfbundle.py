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


def masked_crc32c(data):
    """The checksum BundleEntryProto.crc32c holds: CRC-32C of the tensor bytes, masked as LevelDB
    masks stored CRCs (rotate right 15, add 0xa282ead8).  Pinned against the reference's own index
    files: their optimizer scalars (float32 0.0 decay / momentum, RMSprop rho 0.9 and lr 1e-4, Adadelta
    rho 0.95) carry exactly these values (tests/test_weights_bundle.py)."""
    from . import _lib
    c = _lib.crc32c(data)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


_LISTS = ('variables', 'trainable_variables', 'non_trainable_variables')


def _numbering(items):
    """{list name: [canonical name by index]} for a model whose variables are `items` (weights.spec
    order = Keras Model.variables order: per weighted layer in layer order, the layer's own
    variables -- conv kernel, bias; BN gamma, beta, moving_mean, moving_variance; Bidirectional
    forward then backward kernel, recurrent_kernel, bias).  trainable_variables drops the moving
    statistics, non_trainable_variables keeps only them."""
    names = [n for n, _, _ in items]
    moving = {n for n, _, r in items if r in ('bn_mean', 'bn_var')}
    return {'variables': names,
            'trainable_variables': [n for n in names if n not in moving],
            'non_trainable_variables': [n for n in names if n in moving]}


def layout(shapes):
    """Identify a bundle's model and map its variable keys to canonical ``layer_with_weights-k/var``
    names (``weights.spec``).  -> (kind, n_classes, head, {bundle key: canonical name}).

    A Keras 2.6 SavedModel checkpoint names every variable by the first path a breadth-first walk of
    the object graph reaches it on; the root's children are its layers (``layer_with_weights-k``
    for weighted layers) and then the ``variables`` / ``trainable_variables`` /
    ``non_trainable_variables`` lists the SavedModel serialisation attaches.  Hence two layouts:

    * **base models** (OD ``timit/models/timit{1.0,2.0}``, SI ``timit/model``): every conv / BN /
      Dense variable at depth 2 under its own ``layer_with_weights-k``; the Bidirectional LSTM's
      six tensors sit deeper (``.../forward_layer/cell/kernel``), so they are named by their index
      in one of the lists (timit2.0 ``variables/116..121``, timit1.0 ``trainable_variables/80..85``,
      SI ``trainable_variables/82..87``).
    * **the deployed SI model** that ``transfer_learning`` saves (``speaker_identification.py:401-410,
      456``; loaded by SI ``record_on_pc.py:76-77`` and ``speaker_identification_post_processing.py:
      205-206``): ``Model(inputs, Dense(dim, sigmoid, name='customized_dense')(sliced_base(inputs)))``.
      The root's weighted layers are the nested sliced base model (``layer_with_weights-0``) and
      ``customized_dense`` (``layer_with_weights-1``, kernel [512, dim]).  The base model's variables
      are at depth >= 3 under ``layer_with_weights-0/...``, so the walk names them by their index in
      the root's lists first (depth 2): ``variables/i`` etc., numbered over the nested model's
      variables followed by the head's.  Any that do appear under the nested path are mapped too.
      The head is sigmoid and K = dim.

    Parity against a real TensorFlow save of the deployed model is unpinned (no such file exists in
    the reference; the key layout above is Keras 2.6's checkpoint naming, tested with a committed
    writer of that layout).
    """
    from . import _lib, weights
    top = {k for k in shapes if k.startswith('layer_with_weights-')}
    lww = {int(k.split('/')[0].split('-')[1]) for k in top}
    listed = [k for k in shapes if k.split('/')[0] in _LISTS]
    if lww and max(lww) >= 2:    # a base model: one top-level entry per weighted layer
        k0 = shapes.get('layer_with_weights-0/kernel')
        kind = weights.OD if k0 is not None and len(k0) == 4 else weights.SI
        if kind == weights.OD:
            items, n_classes, head = weights.od_spec(), 2, _lib.HEAD_SOFTMAX
        else:
            head_kernel = shapes.get('layer_with_weights-42/kernel')
            if head_kernel is None or len(head_kernel) != 2:
                raise ValueError('unrecognised bundle layout: an SI base model without its Dense '
                                 'head (layer_with_weights-42/kernel)')
            n_classes = head_kernel[1]
            items = weights.si_spec(n_classes)
            head = _lib.HEAD_SOFTMAX
        mapping = {k: k for k in top}
    else:                        # the deployed transfer-learning model
        if 'layer_with_weights-1/kernel' not in shapes:
            raise ValueError('unrecognised bundle layout: neither a base model nor a '
                             'transfer_learning (nested base + customized_dense) model')
        kind = weights.SI
        if len(shapes['layer_with_weights-1/kernel']) != 2:
            raise ValueError('unrecognised bundle layout: layer_with_weights-1/kernel is not a '
                             'Dense kernel')
        n_classes = shapes['layer_with_weights-1/kernel'][1]
        head = _lib.HEAD_SIGMOID
        items = weights.si_spec(n_classes)
        head_name = items[-2][0].rsplit('/', 1)[0]      # layer_with_weights-42
        mapping = {'layer_with_weights-1/kernel': head_name + '/kernel',
                   'layer_with_weights-1/bias': head_name + '/bias'}
        for k in top:            # base variables the walk reached through the nested model
            if k.startswith('layer_with_weights-0/layer_with_weights-'):
                mapping[k] = k[len('layer_with_weights-0/'):]
    num = _numbering(items)
    for k in listed:
        lst, i = k.split('/')[:2]
        if k.count('/') != 1 or not i.isdigit():
            continue
        if int(i) < len(num[lst]):
            mapping.setdefault(k, num[lst][int(i)])
    want = {n: tuple(sh) for n, sh, _ in items}
    got = {}
    for k, n in list(mapping.items()):
        if n not in want or k not in shapes:
            del mapping[k]
            continue
        if tuple(shapes[k]) != want[n]:
            raise ValueError(f'{k} -> {n}: shape {tuple(shapes[k])} != {want[n]}')
        if n in got:
            raise ValueError(f'{n} stored twice ({got[n]}, {k})')
        got[n] = k
    missing = [n for n in want if n not in got]
    if missing:
        raise ValueError(f'bundle lacks {len(missing)} variables, e.g. {missing[:3]}')
    return kind, n_classes, head, mapping


def canonical_names(shapes, bilstm_layer=None):
    """{bundle key: canonical name} (``layout``; bilstm_layer is implied by the model)."""
    return layout(shapes)[3]


def load_bundle(model_dir, bilstm_layer=None, with_layout=False, verify=True):
    """Read trained weights from ``<model_dir>/variables/variables.{index,data-00000-of-00001}``,
    verifying every tensor's CRC-32C against the index (TF's BundleReader does the same and fails
    with DataLoss).  -> {canonical name: float32 array}, or (weights, (kind, n_classes, head)) with
    ``with_layout``.  Raises FileNotFoundError when the data shard is absent (the reference's case
    today), ValueError on a checksum mismatch or an unrecognised layout."""
    index = os.path.join(model_dir, 'variables', 'variables.index')
    shard = os.path.join(model_dir, 'variables', 'variables.data-00000-of-00001')
    entries = read_index(index)
    if not os.path.exists(shard):
        raise FileNotFoundError(f'{shard} is absent (listed in the reference .MISSING_LARGE_BLOBS)')
    kind, n_classes, head, names = layout(variable_shapes(index))
    out = {}
    with open(shard, 'rb') as f:
        for k, e in entries.items():
            short = k.replace('/.ATTRIBUTES/VARIABLE_VALUE', '')
            if short not in names:
                continue
            f.seek(e['offset'])
            raw = f.read(e['size'])
            if len(raw) != e['size']:
                raise ValueError(f'{shard}: {k} truncated ({len(raw)} of {e["size"]} bytes)')
            if verify and e['crc32c'] is not None and masked_crc32c(raw) != e['crc32c']:
                raise ValueError(f'{shard}: checksum mismatch for {k} (DataLoss)')
            arr = np.frombuffer(raw, dtype=_DTYPES[e['dtype']]).reshape(e['shape'])
            out[names[short]] = arr.astype(np.float32)
    if with_layout:
        return out, (kind, n_classes, head)
    return out
