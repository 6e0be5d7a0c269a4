"""numpy restatement of the two Keras graphs (inference mode) -- TEST INFRASTRUCTURE ONLY.

OD-NET: ``ResLSTM`` (``OverlapDetection/scripts/overlap_detector_temp.py:253-303``), layer graph
as decoded from ``OverlapDetection/timit/models/timit2.0/keras_metadata.pb``.
SI-NET: ``res_model`` + deployed head (``SpeakerIdentification/scripts/speaker_identification.py:
168-218, 401-410``), variable shapes from ``SpeakerIdentification/timit/model/variables/
variables.index``.

Keras 2.6 semantics restated here (TF/Keras is absent from this image: parity *unpinned*):
  * ``padding='same'``: pad_total = max((ceil(in/s)-1)*s + k - in, 0), before = total // 2
    (so kernel 4 pads 1 before / 2 after; MaxPool 'same' pads the end with -inf).
  * BatchNormalization(eps=1e-3) with moving statistics.
  * ELU(alpha=1), ReLU, LeakyReLU(alpha=0.3).
  * LSTM gates i, f, c, o; sigmoid recurrent activation; tanh; h0 = c0 = 0;
    Bidirectional(merge_mode='concat') returns [h_fwd(T-1), h_bwd(after x[0])].
Weights are a dict keyed ``layer_with_weights-<k>/<var>`` (the variables.index names); the
Bidirectional layer's six arrays are keyed ``layer_with_weights-<k>/{forward,backward}/{kernel,
recurrent_kernel,bias}``.
"""
import numpy as np

CHANNELS = (32, 32, 32, 64, 64, 64, 128, 128, 128)
POOL = (True, False, False, True, False, False, True, False, False)
BN_EPS = 1e-3
LEAKY_ALPHA = np.float32(0.3)
OD_INPUT_SHAPE = (128, 151, 3)
STEM_FILTERS = 16
MEAN_AXIS = 1            # Lambda(lambda x: K.mean(x, axis=1)) on NHWC: the mel (H) axis
LSTM_UNITS = 256
OD_DROPOUT = 0.25        # before LeakyReLU; identity at inference
OD_CLASSES = 2
# tests/test_keras_graph.py checks these (and weights.od_spec's kernel shapes) layer by layer
# against the graph in the reference's keras_metadata.pb (tests/golden/od_keras_graph.json)


def _same_pad(n, k, s):
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


def conv2d(x, kernel, bias, stride=1):
    """Keras Conv2D(padding='same') on NHWC; kernel [kh, kw, cin, cout]."""
    kh, kw, cin, cout = kernel.shape
    n, h, w, c = x.shape
    assert c == cin
    ph = _same_pad(h, kh, stride)
    pw = _same_pad(w, kw, stride)
    xp = np.pad(x, ((0, 0), ph, pw, (0, 0)))
    ho = -(-h // stride)
    wo = -(-w // stride)
    out = np.zeros((n, ho, wo, cout), dtype=x.dtype)
    for dy in range(kh):
        for dx in range(kw):
            patch = xp[:, dy:dy + stride * (ho - 1) + 1:stride, dx:dx + stride * (wo - 1) + 1:stride, :]
            out += patch @ kernel[dy, dx].astype(x.dtype)
    return out + bias.astype(x.dtype)


def maxpool2d_same(x, s=2):
    n, h, w, c = x.shape
    ph = _same_pad(h, s, s)
    pw = _same_pad(w, s, s)
    xp = np.pad(x, ((0, 0), ph, pw, (0, 0)), constant_values=-np.inf)
    ho, wo = xp.shape[1] // s, xp.shape[2] // s
    return xp[:, :ho * s, :wo * s].reshape(n, ho, s, wo, s, c).max(axis=(2, 4))


def batchnorm(x, W, k):
    g = W[f'layer_with_weights-{k}/gamma'].astype(x.dtype)
    b = W[f'layer_with_weights-{k}/beta'].astype(x.dtype)
    m = W[f'layer_with_weights-{k}/moving_mean'].astype(x.dtype)
    v = W[f'layer_with_weights-{k}/moving_variance'].astype(x.dtype)
    return (x - m) / np.sqrt(v + BN_EPS) * g + b


def elu(x):
    return np.where(x > 0, x, np.expm1(np.minimum(x, 0)))


def relu(x):
    return np.maximum(x, 0)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_last(x, kernel, rec, bias):
    """Keras LSTM(return_sequences=False) on x [N, T, D] -> h_T [N, units]."""
    n, t, _ = x.shape
    u = rec.shape[0]
    h = np.zeros((n, u), dtype=x.dtype)
    c = np.zeros((n, u), dtype=x.dtype)
    xw = x @ kernel.astype(x.dtype) + bias.astype(x.dtype)
    for s in range(t):
        z = xw[:, s] + h @ rec.astype(x.dtype)
        i = sigmoid(z[:, :u])
        f = sigmoid(z[:, u:2 * u])
        g = np.tanh(z[:, 2 * u:3 * u])
        o = sigmoid(z[:, 3 * u:])
        c = f * c + i * g
        h = o * np.tanh(c)
    return h


def bilstm(x, W, k):
    p = f'layer_with_weights-{k}'
    hf = lstm_last(x, W[p + '/forward/kernel'], W[p + '/forward/recurrent_kernel'], W[p + '/forward/bias'])
    hb = lstm_last(x[:, ::-1], W[p + '/backward/kernel'], W[p + '/backward/recurrent_kernel'], W[p + '/backward/bias'])
    return np.concatenate([hf, hb], axis=1)


def softmax(z):
    z = z - z.max(axis=1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=1, keepdims=True)


def _conv(x, W, k, stride=1):
    return conv2d(x, W[f'layer_with_weights-{k}/kernel'], W[f'layer_with_weights-{k}/bias'], stride)


def od_forward(x, W, dtype=np.float64, return_logits=False):
    """OD-NET predict: x float [N,128,151,3] (PNG values 0..255) -> softmax probs [N,2]."""
    x = np.asarray(x, dtype=dtype)
    net = _conv(x, W, 0)
    k = 1
    for c, pool in zip(CHANNELS, POOL):
        res = net
        out = elu(batchnorm(net, W, k))
        out = _conv(out, W, k + 1)
        out = elu(batchnorm(out, W, k + 2))
        out = _conv(out, W, k + 3)
        if pool:
            res = _conv(net, W, k + 4, stride=2)
            out = maxpool2d_same(out)
            k += 5
        else:
            k += 4
        net = res + out
    assert k == 40
    seq = net.mean(axis=MEAN_AXIS)                           # Lambda(K.mean(x, axis=1)) -> [N,19,128]
    h = bilstm(seq, W, 40)
    h = np.where(h > 0, h, h * dtype(LEAKY_ALPHA))           # Dropout no-op, LeakyReLU(0.3)
    z = h @ W['layer_with_weights-41/kernel'].astype(dtype) + W['layer_with_weights-41/bias'].astype(dtype)
    return z if return_logits else softmax(z)


def conv1d(x, kernel, bias, stride=1):
    """Keras Conv1D(padding='same') on [N,T,C]; kernel [k, cin, cout]."""
    return conv2d(x[:, :, None, :], kernel[:, None], bias, stride)[:, :, 0, :]


def maxpool1d_same(x):
    return maxpool2d_same(x[:, :, None, :])[:, :, 0, :] if x.shape[1] % 2 == 0 else \
        maxpool2d_same(np.concatenate([x[:, :, None, :], x[:, :, None, :]], axis=2))[:, :, 0, :]


def _conv1(x, W, k, stride=1):
    return conv1d(x, W[f'layer_with_weights-{k}/kernel'], W[f'layer_with_weights-{k}/bias'], stride)


def si_forward(x, W, head='softmax', dtype=np.float64, return_logits=False):
    """SI-NET predict: x [N,256,39] -> [N,K] (softmax base model, or sigmoid deployed head)."""
    x = np.asarray(x, dtype=dtype)
    net = _conv1(x, W, 0)
    k = 1
    for c, pool in zip(CHANNELS, POOL):
        res = net
        inp = net
        if pool:
            inp = maxpool1d_same(net)
        out = relu(batchnorm(inp, W, k))
        out = _conv1(out, W, k + 1)
        out = relu(batchnorm(out, W, k + 2))
        if pool:
            res = _conv1(net, W, k + 3, stride=2)
            out = _conv1(out, W, k + 4)
            k += 5
        else:
            out = _conv1(out, W, k + 3)
            k += 4
        net = res + out
    assert k == 40
    net = relu(batchnorm(net, W, 40))                      # final BN -> ReLU -> Dropout(no-op)
    n, t, c = net.shape
    net = net[:, :t // 4 * 4].reshape(n, t // 4, 4, c).mean(axis=2)   # AveragePooling1D(4)
    h = bilstm(net, W, 41)
    z = h @ W['layer_with_weights-42/kernel'].astype(dtype) + W['layer_with_weights-42/bias'].astype(dtype)
    if return_logits:
        return z
    return softmax(z) if head == 'softmax' else sigmoid(z)
