"""TEST INFRASTRUCTURE: a writer of TensorFlow tensor bundles (``variables/variables.index`` +
``variables.data-00000-of-00001``) in the key layouts a Keras 2.6 SavedModel uses, so that the
drop-in's reader (``mmla_audio_amd.tfbundle``) can be tested on complete bundles -- the reference
ships only the index files (``.MISSING_LARGE_BLOBS``).

Format written (the reader's docstring has the references): one uncompressed LevelDB data block
(restart at every entry) holding the empty-key BundleHeaderProto and one BundleEntryProto per
tensor in key order, an index block, an empty metaindex block, each followed by the 5-byte trailer
(type 0 + masked CRC-32C of contents + type), and the 48-byte footer.  Tensors are stored
little-endian at 8-byte-aligned offsets of the data shard with their masked CRC-32C.

Layouts (``tfbundle.layout`` explains why Keras names the variables so):
* ``base_keys``: the reference base models -- ``layer_with_weights-k/<var>`` for conv / BN /
  Dense, the Bidirectional LSTM by its index in one of the root's variable lists;
* ``deployed_keys``: ``transfer_learning``'s saved model -- ``layer_with_weights-1/{kernel,bias}``
  = customized_dense, the nested base model's variables by their indices in the root's lists
  (``variables`` / ``trainable_variables`` / ``non_trainable_variables``), optionally some under the
  nested path ``layer_with_weights-0/...``.
A real TensorFlow save of the deployed model does not exist anywhere in the reference, so the
deployed layout's parity with TF itself is unpinned; the base layout's list indices are the ones
the reference's own index files hold (tests/test_weights_bundle.py).
"""
import os
import struct

import numpy as np

from mmla_audio_amd import tfbundle, weights

_DTYPE = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3,
          np.dtype(np.int64): 9}
_MAGIC = 0xdb4775248b80fb57
SUFFIX = '/.ATTRIBUTES/VARIABLE_VALUE'


def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num, wire, payload):
    tag = _varint((num << 3) | wire)
    if wire == 0:
        return tag + _varint(payload)
    if wire == 2:
        return tag + _varint(len(payload)) + payload
    if wire == 5:
        return tag + struct.pack('<I', payload)
    raise ValueError(wire)


def _entry_proto(dtype, shape, offset, size, crc):
    dims = b''.join(_field(2, 2, _field(1, 0, d)) for d in shape)
    out = _field(1, 0, dtype) + _field(2, 2, dims)
    if offset:
        out += _field(4, 0, offset)
    out += _field(5, 0, size) + _field(6, 5, crc)
    return out


def _block(entries):
    body = bytearray()
    restarts = []
    for k, v in entries:
        restarts.append(len(body))
        body += _varint(0) + _varint(len(k)) + _varint(len(v)) + k + v
    if not restarts:
        restarts = [0]
    for r in restarts:
        body += struct.pack('<I', r)
    body += struct.pack('<I', len(restarts))
    return bytes(body)


def _trailer(block):
    return b'\x00' + struct.pack('<I', tfbundle.masked_crc32c(block + b'\x00'))


def write_bundle(model_dir, tensors):
    """tensors: {bundle key (without the .ATTRIBUTES suffix): ndarray} -> a complete bundle under
    model_dir/variables/."""
    d = os.path.join(model_dir, 'variables')
    os.makedirs(d, exist_ok=True)
    data = bytearray()
    entries = []
    for key in sorted(tensors):
        a = np.ascontiguousarray(tensors[key])
        raw = a.astype(a.dtype.newbyteorder('<')).tobytes()
        off = (len(data) + 7) // 8 * 8
        data += b'\0' * (off - len(data))
        data += raw
        full = (key + SUFFIX).encode()
        entries.append((full, _entry_proto(_DTYPE[a.dtype], a.shape, off, len(raw),
                                           tfbundle.masked_crc32c(raw))))
    header = _field(1, 0, 1) + _field(3, 2, _field(1, 0, 1))   # num_shards 1, version.producer 1
    entries = [(b'', header)] + sorted(entries)
    out = bytearray()
    blk = _block(entries)
    data_handle = (len(out), len(blk))
    out += blk + _trailer(blk)
    meta = _block([])
    meta_handle = (len(out), len(meta))
    out += meta + _trailer(meta)
    idx = _block([(entries[-1][0], _varint(data_handle[0]) + _varint(data_handle[1]))])
    idx_handle = (len(out), len(idx))
    out += idx + _trailer(idx)
    foot = _varint(meta_handle[0]) + _varint(meta_handle[1]) + _varint(idx_handle[0]) + _varint(idx_handle[1])
    out += foot + b'\0' * (40 - len(foot)) + struct.pack('<Q', _MAGIC)
    with open(os.path.join(d, 'variables.index'), 'wb') as f:
        f.write(bytes(out))
    with open(os.path.join(d, 'variables.data-00000-of-00001'), 'wb') as f:
        f.write(bytes(data))


def _lists(items):
    return tfbundle._numbering(items)


def base_keys(kind, W, lstm_list='variables', n_classes=None):
    """{bundle key: array} for a base model: top-level layer keys + the LSTM by list index"""
    items = weights.spec(kind, n_classes)
    num = _lists(items)
    out = {}
    for n, _, r in items:
        if r.startswith('lstm'):
            out[f'{lstm_list}/{num[lstm_list].index(n)}'] = W[n]
        else:
            out[n] = W[n]
    return out


def deployed_keys(W, n_classes, trainable_first=False, nested=()):
    """{bundle key: array} for transfer_learning's saved SI model with a K = n_classes head.
    trainable_first: trainable base variables under trainable_variables/j, the BN moving
    statistics under variables/i (else every base variable under variables/i); nested: canonical
    base names stored under layer_with_weights-0/<name> instead."""
    items = weights.si_spec(n_classes)
    head = items[-2][0].rsplit('/', 1)[0]
    num = _lists(items)
    out = {'layer_with_weights-1/kernel': W[head + '/kernel'], 'layer_with_weights-1/bias': W[head + '/bias']}
    for n, _, r in items[:-2]:
        if n in nested:
            out['layer_with_weights-0/' + n] = W[n]
        elif trainable_first and r not in ('bn_mean', 'bn_var'):
            out[f'trainable_variables/{num["trainable_variables"].index(n)}'] = W[n]
        else:
            out[f'variables/{num["variables"].index(n)}'] = W[n]
    # what a Keras save also holds and the reader must skip: optimizer slots, metrics, counters
    out['optimizer/iter'] = np.array(1234, np.int64)
    out['optimizer/learning_rate'] = np.array(1e-6, np.float32)
    out['optimizer/layer_with_weights-1/kernel/.OPTIMIZER_SLOT/rms'] = np.zeros_like(W[head + '/kernel'])
    out['keras_api/metrics/0/total'] = np.array(3.0, np.float32)
    out['save_counter'] = np.array(1, np.int64)
    return out
