"""Weight layouts of the two reference networks, seeded synthetic weights, and packing for the C-ABI.

The trained weights are absent from the reference (``.MISSING_LARGE_BLOBS:1-6``), so parity runs on
seeded synthetic weights laid out exactly like the reference ``variables.index`` files
(SURVEY.md 8a "Weight layouts").  ``mmla_audio_amd.tfbundle.load_bundle`` loads the real ones the
moment the data shard is supplied.

Canonical names are the bundle's ``layer_with_weights-<k>/<var>``; the Bidirectional LSTM's six
tensors are ``layer_with_weights-<k>/{forward,backward}/{kernel,recurrent_kernel,bias}``.

OD (``OverlapDetection/timit/models/timit2.0``): lww-0 stem Conv2D [1,1,3,16]; per res_block
``BN, Conv3x3, BN, Conv(4,1)[, shortcut Conv1x1/2]`` through lww-39; lww-40 BiLSTM(256) on 128
inputs; lww-41 Dense [512,2].
SI (``SpeakerIdentification/timit/model``): lww-0 Conv1D [4,39,32]; per res_unit
``BN, Conv3, BN[, shortcut Conv1/2], Conv3`` through lww-39; lww-40 final BN128; lww-41 BiLSTM;
lww-42 Dense [512,K] (K=630 softmax base model, or the deployed ``customized_dense`` sigmoid head,
``speaker_identification.py:409``).

The packed order handed to ``mmla_load_weights`` is the order of ``spec()``: ascending layer index;
conv/dense = kernel, bias; BN = gamma, beta, moving_mean, moving_variance; BiLSTM = forward kernel,
recurrent_kernel, bias, backward kernel, recurrent_kernel, bias.  Arrays keep the Keras layouts
(Conv2D [kh,kw,cin,cout], Conv1D [k,cin,cout], Dense [in,out], LSTM [in,4u] gates i,f,c,o).
"""
import numpy as np

OD = 0
SI = 1
CHANNELS = (32, 32, 32, 64, 64, 64, 128, 128, 128)
POOL = (True, False, False, True, False, False, True, False, False)
LSTM_UNITS = 256


def _bn(k, c):
    p = f'layer_with_weights-{k}/'
    return [(p + 'gamma', (c,), 'bn_gamma'), (p + 'beta', (c,), 'bn_beta'),
            (p + 'moving_mean', (c,), 'bn_mean'), (p + 'moving_variance', (c,), 'bn_var')]


def _conv(k, shape):
    p = f'layer_with_weights-{k}/'
    return [(p + 'kernel', tuple(shape), 'kernel'), (p + 'bias', (shape[-1],), 'bias')]


def _bilstm(k, d):
    out = []
    for side in ('forward', 'backward'):
        p = f'layer_with_weights-{k}/{side}/'
        out += [(p + 'kernel', (d, 4 * LSTM_UNITS), 'lstm_kernel'),
                (p + 'recurrent_kernel', (LSTM_UNITS, 4 * LSTM_UNITS), 'lstm_rec'),
                (p + 'bias', (4 * LSTM_UNITS,), 'lstm_bias')]
    return out


def od_spec():
    """[(name, shape, role)] in packed order for OD-NET."""
    s = _conv(0, (1, 1, 3, 16))
    k = 1
    cin = 16
    for c, pool in zip(CHANNELS, POOL):
        s += _bn(k, cin) + _conv(k + 1, (3, 3, cin, c)) + _bn(k + 2, c) + _conv(k + 3, (4, 1, c, c))
        if pool:
            s += _conv(k + 4, (1, 1, cin, c))
            k += 5
        else:
            k += 4
        cin = c
    s += _bilstm(40, 128)
    s += _conv(41, (512, 2))
    return s


def si_spec(n_classes=630):
    """[(name, shape, role)] in packed order for SI-NET with a K-way head."""
    s = _conv(0, (4, 39, 32))
    k = 1
    cin = 32
    for c, pool in zip(CHANNELS, POOL):
        s += _bn(k, cin) + _conv(k + 1, (3, cin, c)) + _bn(k + 2, c)
        if pool:
            s += _conv(k + 3, (1, cin, c)) + _conv(k + 4, (3, c, c))
            k += 5
        else:
            s += _conv(k + 3, (3, c, c))
            k += 4
        cin = c
    s += _bn(40, 128)
    s += _bilstm(41, 128)
    s += _conv(42, (512, n_classes))
    return s


def spec(kind, n_classes=None):
    if kind == OD:
        return od_spec()
    return si_spec(630 if n_classes is None else n_classes)


def _glorot(rng, shape):
    if len(shape) == 2:
        fan_in, fan_out = shape
    else:
        rf = int(np.prod(shape[:-2]))
        fan_in, fan_out = rf * shape[-2], rf * shape[-1]
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=shape), fan_in, lim * lim / 3.0


def _orthogonal(rng, shape):
    a = rng.standard_normal((shape[1], shape[0]))
    q, r = np.linalg.qr(a)
    q = q * np.sign(np.diag(r))
    return q.T


SI_HEAD_GAIN = 10.0   # synthetic SI Dense kernel scale: decisive argmax at K = 630 (logit std ~4)


def synthetic(kind, seed=0, n_classes=None, head_gain=None):
    """Seeded synthetic weights in the reference layout.

    Kernels are Glorot-uniform (the Keras default the reference trains from), recurrent kernels
    orthogonal, LSTM biases ``unit_forget_bias``.  BatchNorm moving statistics are not the
    Keras initial (0, 1): they are set from a second-moment estimate propagated through the graph
    so that every BN actually normalises, as a trained model's would, and the stem kernel is scaled
    for the input range (0..255 PNG values for OD, MFCC magnitudes for SI).  All non-zero, so every
    fused bias / BN / residual term is exercised by parity tests.  The SI head's Dense kernel is
    scaled by ``head_gain`` (default SI_HEAD_GAIN): Glorot alone gives logits with std ~0.4 over 630
    classes, a nearly flat softmax a trained classifier would not produce and on which argmax checks
    decide little.
    """
    rng = np.random.default_rng(np.random.PCG64(0x6D6D6C61 + 7919 * seed + 31 * kind))
    W = {}
    m2 = 2.0e4 if kind == OD else 150.0     # second moment of the network input
    stem_gain = None
    act_m2 = 0.6                              # E[act(bn(x))^2] for unit-variance BN output
    items = spec(kind, n_classes)
    i = 0
    cur = m2
    resid = None
    while i < len(items):
        name, shape, role = items[i]
        if role == 'kernel':
            w, fan_in, var_w = _glorot(rng, shape)
            if stem_gain is None:
                stem_gain = 1.0 / np.sqrt(fan_in * var_w * m2)
                w = w * stem_gain
                var_w = var_w * stem_gain ** 2
            W[name] = w
            b_name = items[i + 1][0]
            W[b_name] = rng.uniform(-0.05, 0.05, size=items[i + 1][1])
            cur = fan_in * var_w * cur + 0.05 ** 2 / 3
            i += 2
            continue
        if role == 'bn_gamma':
            c = shape[0]
            W[name] = rng.uniform(0.8, 1.2, size=c)
            W[items[i + 1][0]] = rng.uniform(-0.1, 0.1, size=c)
            mean = rng.uniform(-0.1, 0.1, size=c) * np.sqrt(cur)
            W[items[i + 2][0]] = mean
            W[items[i + 3][0]] = cur * rng.uniform(0.8, 1.25, size=c)
            cur = act_m2
            i += 4
            continue
        if role == 'lstm_kernel':
            for j in range(2):
                kn, ks, _ = items[i + 3 * j]
                rn, rs, _ = items[i + 3 * j + 1]
                bn, bs, _ = items[i + 3 * j + 2]
                W[kn] = _glorot(rng, ks)[0]
                W[rn] = _orthogonal(rng, rs)
                b = rng.uniform(-0.05, 0.05, size=bs)
                b[LSTM_UNITS:2 * LSTM_UNITS] += 1.0
                W[bn] = b
            i += 6
            continue
        raise AssertionError(f'unexpected role {role} at {name}')
    del resid
    if head_gain is None:
        head_gain = SI_HEAD_GAIN if kind == SI else 1.0
    head = [n for n, _, r in items if r == 'kernel'][-1]
    W[head] = W[head] * head_gain
    return {k: np.asarray(v, dtype=np.float32) for k, v in W.items()}


def check(kind, W, n_classes=None):
    """Raise ValueError unless W has exactly the spec's names and shapes."""
    items = spec(kind, n_classes)
    names = {n for n, _, _ in items}
    missing = [n for n in names if n not in W]
    if missing:
        raise ValueError(f'missing weights: {missing[:5]}...')
    for n, s, _ in items:
        if tuple(W[n].shape) != tuple(s):
            raise ValueError(f'{n}: shape {tuple(W[n].shape)} != expected {s}')


def pack(kind, W, n_classes=None):
    """Flatten W into the canonical float32 blob for ``mmla_load_weights``."""
    check(kind, W, n_classes)
    return np.concatenate([np.ascontiguousarray(W[n], dtype=np.float32).ravel()
                           for n, _, _ in spec(kind, n_classes)])


def n_params(kind, n_classes=None):
    return int(sum(int(np.prod(s)) for _, s, _ in spec(kind, n_classes)))
