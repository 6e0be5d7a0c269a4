"""CPU: the OD-NET restatement (oracle/nets.py constants + the weight layout of
mmla_audio_amd/weights.py, which both the oracle and the HIP path consume) against the layer graph
the reference ships in OverlapDetection/timit/models/timit{1.0,2.0}/keras_metadata.pb, extracted
into tests/golden/od_keras_graph.json by tests/golden/make_keras_graph.py.

Checked layer by layer: class, kernel sizes, strides, padding, activations, BatchNormalization
epsilon, MaxPooling, Add connectivity, the Lambda's mean axis, Bidirectional(LSTM) units /
activations / merge mode, Dropout, LeakyReLU alpha, Dense head -- and that the order of the
layers with weights (Keras `layer_with_weights-k`) and their shapes equal weights.od_spec().
"""
import json
import os

import numpy as np
import pytest

from mmla_audio_amd import weights
from oracle import nets

GRAPH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'od_keras_graph.json')


@pytest.fixture(scope='module')
def graphs():
    return json.load(open(GRAPH))


def expected_ops():
    """canonical op list of OD-NET as oracle/nets.py computes it (kernel sizes from od_spec)"""
    spec = [s for s in weights.od_spec() if s[2] == 'kernel']
    ks = iter(s[1] for s in spec)
    ops = []

    def op(cls, params, *inputs):
        ops.append((cls, params, inputs))
        return len(ops) - 1

    def conv(x, filters, stride=1):
        k = next(ks)
        assert k[-1] == filters
        return op('Conv2D', (filters, tuple(k[:2]), (stride, stride), 'same', 'linear'), x)

    x = op('InputLayer', (None,) + nets.OD_INPUT_SHAPE)
    net = conv(x, nets.STEM_FILTERS)
    for c, pool in zip(nets.CHANNELS, nets.POOL):
        out = op('Activation', ('elu',), op('BatchNormalization', (nets.BN_EPS,), net))
        out = conv(out, c)
        out = op('Activation', ('elu',), op('BatchNormalization', (nets.BN_EPS,), out))
        out = conv(out, c)
        if pool:
            sc = conv(net, c, 2)
            out = op('MaxPooling2D', ((2, 2), (2, 2), 'same'), out)
            net = op('Add', (), sc, out)
        else:
            net = op('Add', (), net, out)
    seq = op('Lambda', ('mean', nets.MEAN_AXIS), net)
    h = op('Bidirectional', ('LSTM', nets.LSTM_UNITS, 'tanh', 'sigmoid', False, 'concat'), seq)
    h = op('Dropout', (nets.OD_DROPOUT,), h)
    h = op('LeakyReLU', (float(nets.LEAKY_ALPHA),), h)
    assert next(ks) == (2 * nets.LSTM_UNITS, nets.OD_CLASSES)
    op('Dense', (nets.OD_CLASSES, 'softmax'), h)
    assert next(ks, None) is None
    return ops


def keras_ops(g):
    """the same canonical form read from the reference's Keras JSON"""
    ids, ops = {}, []
    for l in g['layers']:
        c = l['class']
        if c == 'InputLayer':
            p = tuple(l['batch_input_shape'])
        elif c == 'Conv2D':
            p = (l['filters'], tuple(l['kernel_size']), tuple(l['strides']), l['padding'], l['activation'])
        elif c == 'BatchNormalization':
            p = (l['epsilon'],)
        elif c == 'Activation':
            p = (l['activation'],)
        elif c == 'MaxPooling2D':
            p = (tuple(l['pool_size']), tuple(l['strides']), l['padding'])
        elif c == 'Add':
            p = ()
        elif c == 'Lambda':
            refs = l['function_refs']
            assert {'K', 'mean', 'axis'} <= set(refs['identifiers'])
            axes = [i for i in refs['small_int_constants'] if i != 0]
            p = ('mean', axes[0] if len(axes) == 1 else tuple(axes))
        elif c == 'Bidirectional':
            L = l['layer']
            assert L['use_bias'] and L['unit_forget_bias'] and not L['go_backwards']
            assert L['dropout'] == 0 and L['recurrent_dropout'] == 0
            p = (L['class'], L['units'], L['activation'], L['recurrent_activation'],
                 L['return_sequences'], l['merge_mode'])
        elif c == 'Dropout':
            p = (l['rate'],)
        elif c == 'LeakyReLU':
            p = (l['alpha'],)
        elif c == 'Dense':
            p = (l['units'], l['activation'])
        else:
            raise AssertionError(f'unexpected layer class {c}')
        ids[l['name']] = len(ops)
        ops.append((c, p, tuple(ids[n] for n in l['inbound'])))
    return ops


@pytest.mark.parametrize('model', ['timit1.0', 'timit2.0'])
def test_graph_matches_restatement(graphs, model):
    g = graphs[model]
    assert g['keras_version'] == '2.6.0' and g['output_layers'] == ['dense']
    got, want = keras_ops(g), expected_ops()
    assert len(got) == len(want)
    for i, (a, b) in enumerate(zip(got, want)):
        assert a == b, f'{model} layer {i} ({g["layers"][i]["name"]}): keras {a} != restatement {b}'


def test_two_models_share_architecture(graphs):
    assert keras_ops(graphs['timit1.0']) == keras_ops(graphs['timit2.0'])


def test_weighted_layer_order_matches_spec(graphs):
    """layer_with_weights-k = k-th layer with variables in model order: its class and shapes must
    be those of weights.od_spec() group k (channels propagated through the graph)"""
    g = graphs['timit2.0']
    ch = {}
    groups = {}
    for name, shape, role in weights.od_spec():
        groups.setdefault(int(name.split('/')[0].split('-')[1]), []).append((name, shape, role))
    k = 0
    for l in g['layers']:
        c = l['class']
        cin = ch[l['inbound'][0]] if l['inbound'] else l['batch_input_shape'][-1]
        if c == 'Conv2D':
            grp = groups[k]
            assert [r for _, _, r in grp] == ['kernel', 'bias']
            assert grp[0][1] == tuple(l['kernel_size']) + (cin, l['filters']), l['name']
            k += 1
            ch[l['name']] = l['filters']
        elif c == 'BatchNormalization':
            grp = groups[k]
            assert [r for _, _, r in grp] == ['bn_gamma', 'bn_beta', 'bn_mean', 'bn_var']
            assert all(s == (cin,) for _, s, _ in grp), l['name']
            k += 1
            ch[l['name']] = cin
        elif c == 'Bidirectional':
            grp = groups[k]
            u = l['layer']['units']
            assert [s for _, s, _ in grp] == [(cin, 4 * u), (u, 4 * u), (4 * u,)] * 2
            k += 1
            ch[l['name']] = 2 * u
        elif c == 'Dense':
            assert groups[k][0][1] == (cin, l['units'])
            k += 1
            ch[l['name']] = l['units']
        elif c == 'Add':
            assert len({ch[n] for n in l['inbound']}) == 1
            ch[l['name']] = cin
        else:
            ch[l['name']] = cin
    assert k == len(groups) == 42


def test_leaky_alpha_is_float32(graphs):
    alpha = [l['alpha'] for l in graphs['timit2.0']['layers'] if l['class'] == 'LeakyReLU'][0]
    assert np.float32(alpha) == nets.LEAKY_ALPHA and alpha == float(nets.LEAKY_ALPHA)
