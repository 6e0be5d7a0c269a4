"""CPU: weight layouts vs the reference's own variables.index files (copied data fixtures)."""
import os

import numpy as np
import pytest

from mmla_audio_amd import tfbundle, weights

G = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.mark.parametrize('fname,kind,bilstm,ncls', [
    ('od_timit2.0_variables.index', weights.OD, 40, None),
    ('od_timit1.0_variables.index', weights.OD, 40, None),
    ('si_timit_variables.index', weights.SI, 41, 630),
])
def test_spec_matches_reference_index(fname, kind, bilstm, ncls):
    shapes = tfbundle.variable_shapes(os.path.join(G, fname))
    names = tfbundle.canonical_names(shapes, bilstm)
    got = {names[k]: tuple(v) for k, v in shapes.items() if k in names}
    want = {n: tuple(s) for n, s, _ in weights.spec(kind, ncls)}
    assert got == want


def test_synthetic_is_deterministic_and_packs():
    a = weights.synthetic(weights.OD, seed=3)
    b = weights.synthetic(weights.OD, seed=3)
    pa, pb = weights.pack(weights.OD, a), weights.pack(weights.OD, b)
    assert pa.dtype == np.float32 and np.array_equal(pa, pb)
    assert pa.size == weights.n_params(weights.OD)
    s8 = weights.synthetic(weights.SI, seed=1, n_classes=8)
    assert weights.pack(weights.SI, s8, 8).size == weights.n_params(weights.SI, 8)


def test_missing_data_shard_raises(tmp_path):
    d = tmp_path / 'm' / 'variables'
    d.mkdir(parents=True)
    (d / 'variables.index').write_bytes(open(os.path.join(G, 'od_timit2.0_variables.index'), 'rb').read())
    with pytest.raises(FileNotFoundError):
        tfbundle.load_bundle(str(tmp_path / 'm'), 40)


def test_bundle_roundtrip(tmp_path):
    """Write a data shard laid out at the index's offsets and read it back."""
    idx = os.path.join(G, 'od_timit2.0_variables.index')
    ent = tfbundle.read_index(idx)
    total = max(e['offset'] + e['size'] for e in ent.values())
    blob = np.random.default_rng(0).standard_normal(total // 4 + 1).astype(np.float32).tobytes()[:total]
    d = tmp_path / 'm' / 'variables'
    d.mkdir(parents=True)
    (d / 'variables.index').write_bytes(open(idx, 'rb').read())
    (d / 'variables.data-00000-of-00001').write_bytes(blob)
    W = tfbundle.load_bundle(str(tmp_path / 'm'), 40)
    weights.check(weights.OD, W)
    e = ent['layer_with_weights-2/kernel/.ATTRIBUTES/VARIABLE_VALUE']
    want = np.frombuffer(blob[e['offset']:e['offset'] + e['size']], np.float32).reshape(3, 3, 16, 32)
    assert np.array_equal(W['layer_with_weights-2/kernel'], want)
