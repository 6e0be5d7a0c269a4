"""Extract the OD-NET layer graph from the reference's keras_metadata.pb files into a fixture.

Run in the build container (it reads /root/reference, which the GPU box does not have):
    python tests/golden/make_keras_graph.py
-> tests/golden/od_keras_graph.json: for OverlapDetection/timit/models/timit{1.0,2.0}/keras_metadata.pb
(Keras 2.6 SavedMetadata protobuf; the root node's metadata is the model's Keras JSON) the layer
list in model order with class, name, inbound layer names and the configuration fields the
restatement depends on (kernel sizes, strides, padding, activations, BN epsilon, LeakyReLU alpha,
pooling, LSTM units/activations/merge mode, dropout rates).  The Lambda layer's marshalled
function is not copied: only the identifiers and small integer constants it references are
recorded (the fixture is data, not code).  tests/test_keras_graph.py checks oracle/nets.py and
mmla_audio_amd/weights.py against it.
"""
import base64
import json
import os
import re

REF = '/root/reference/OverlapDetection/timit/models'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'od_keras_graph.json')
KEEP = ('filters', 'kernel_size', 'strides', 'padding', 'activation', 'use_bias', 'epsilon',
        'momentum', 'center', 'scale', 'axis', 'alpha', 'units', 'pool_size', 'rate', 'merge_mode',
        'data_format', 'dilation_rate', 'groups', 'batch_input_shape')


def _varint(b, i):
    r = s = 0
    while True:
        x = b[i]
        i += 1
        r |= (x & 0x7f) << s
        s += 7
        if not x & 0x80:
            return r, i


def _fields(b):
    """protobuf wire-format fields (number, value) of one message"""
    i = 0
    while i < len(b):
        key, i = _varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 2:
            n, i = _varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 5:
            v, i = b[i:i + 4], i + 4
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        else:
            raise ValueError(f'wire type {wt}')
        yield f, v


def _plain(v):
    if isinstance(v, dict) and v.get('class_name') == '__tuple__':
        return [_plain(x) for x in v['items']]
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_plain(x) for x in v]
    return v


def _lambda_tokens(fn):
    """identifiers and small int constants referenced by a marshalled (Python 3.x) lambda"""
    raw = base64.b64decode(fn['items'][0])
    names = set()
    for m in re.finditer(rb'[\x5a\x7a\xda\xfa]([\x01-\x40])', raw):   # short ASCII strings
        n = m.group(1)[0]
        s = raw[m.end():m.end() + n]
        if len(s) == n and re.fullmatch(rb'[A-Za-z_][A-Za-z0-9_]*', s):
            names.add(s.decode())
    ints = sorted({int.from_bytes(raw[m.end():m.end() + 4], 'little', signed=True)
                   for m in re.finditer(rb'[\x69\xe9]', raw)
                   if m.end() + 4 <= len(raw) and
                   -16 <= int.from_bytes(raw[m.end():m.end() + 4], 'little', signed=True) <= 16})
    return {'identifiers': sorted(names), 'small_int_constants': ints}


def model_graph(path):
    data = open(path, 'rb').read()
    for _, node in _fields(data):
        for _, v in _fields(node):
            if isinstance(v, bytes) and v[:1] == b'{':
                j = json.loads(v)
                cfg = j.get('config')
                if isinstance(cfg, dict) and 'layers' in cfg:
                    layers = []
                    for l in cfg['layers']:
                        c = l['config']
                        e = {'class': l['class_name'], 'name': c['name'],
                             'inbound': [x[0] for x in l['inbound_nodes'][0]] if l['inbound_nodes'] else []}
                        e.update({k: _plain(c[k]) for k in KEEP if k in c})
                        if l['class_name'] == 'Bidirectional':
                            inner = c['layer']['config']
                            e['layer'] = {'class': c['layer']['class_name'],
                                          **{k: _plain(inner[k]) for k in (
                                              'units', 'activation', 'recurrent_activation', 'use_bias',
                                              'unit_forget_bias', 'return_sequences', 'go_backwards',
                                              'dropout', 'recurrent_dropout') if k in inner}}
                        if l['class_name'] == 'Lambda':
                            e['function_type'] = c.get('function_type')
                            e['function_refs'] = _lambda_tokens(c['function'])
                        layers.append(e)
                    return {'keras_version': j.get('keras_version'), 'backend': j.get('backend'),
                            'output_layers': [x[0] for x in cfg.get('output_layers', [])],
                            'layers': layers}
    raise ValueError(f'{path}: no model config found')


def main():
    out = {f'timit{v}': model_graph(os.path.join(REF, f'timit{v}', 'keras_metadata.pb'))
           for v in ('1.0', '2.0')}
    json.dump(out, open(OUT, 'w'), indent=1)
    print(OUT, {k: len(v['layers']) for k, v in out.items()})


if __name__ == '__main__':
    main()
