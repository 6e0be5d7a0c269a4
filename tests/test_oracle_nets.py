"""CPU: the numpy net oracle against an independent torch-CPU restatement (two CPU oracles)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mmla_audio_amd import weights
from oracle import nets


def _t(a):
    return torch.as_tensor(np.asarray(a, np.float64))


def _conv_t(x, W, k, stride=1):
    ker = _t(W[f'layer_with_weights-{k}/kernel'])      # [kh,kw,cin,cout]
    kh, kw = ker.shape[:2]
    h, w = x.shape[2], x.shape[3]
    def pads(n, kk, s):
        out = -(-n // s)
        tot = max((out - 1) * s + kk - n, 0)
        return tot // 2, tot - tot // 2
    ph, pw = pads(h, kh, stride), pads(w, kw, stride)
    xp = F.pad(x, (pw[0], pw[1], ph[0], ph[1]))
    return F.conv2d(xp, ker.permute(3, 2, 0, 1), _t(W[f'layer_with_weights-{k}/bias']), stride=stride)


def _bn_t(x, W, k):
    g, b, m, v = (_t(W[f'layer_with_weights-{k}/{n}']) for n in ('gamma', 'beta', 'moving_mean', 'moving_variance'))
    return F.batch_norm(x, m, v, g, b, False, 0.0, 1e-3)


def _lstm_t(x, W, p):
    lstm = torch.nn.LSTM(x.shape[-1], 256, batch_first=True, bidirectional=True).double()
    def reorder(a):   # keras i,f,c,o -> torch i,f,g,o (same order)
        return a
    with torch.no_grad():
        lstm.weight_ih_l0.copy_(_t(W[p + '/forward/kernel']).T)
        lstm.weight_hh_l0.copy_(_t(W[p + '/forward/recurrent_kernel']).T)
        lstm.bias_ih_l0.copy_(_t(W[p + '/forward/bias']))
        lstm.bias_hh_l0.zero_()
        lstm.weight_ih_l0_reverse.copy_(_t(W[p + '/backward/kernel']).T)
        lstm.weight_hh_l0_reverse.copy_(_t(W[p + '/backward/recurrent_kernel']).T)
        lstm.bias_ih_l0_reverse.copy_(_t(W[p + '/backward/bias']))
        lstm.bias_hh_l0_reverse.zero_()
        out, _ = lstm(x)
    return torch.cat([out[:, -1, :256], out[:, 0, 256:]], dim=1)


def od_torch(x, W):
    x = _t(x).permute(0, 3, 1, 2)
    net = _conv_t(x, W, 0)
    k = 1
    for pool in nets.POOL:
        out = _conv_t(F.elu(_bn_t(net, W, k)), W, k + 1)
        out = _conv_t(F.elu(_bn_t(out, W, k + 2)), W, k + 3)
        if pool:
            res = _conv_t(net, W, k + 4, 2)
            h, w = out.shape[2], out.shape[3]
            out = F.max_pool2d(F.pad(out, (0, w % 2, 0, h % 2), value=-np.inf), 2)
            k += 5
        else:
            res = net
            k += 4
        net = res + out
    seq = net.mean(dim=2).permute(0, 2, 1)
    h = F.leaky_relu(_lstm_t(seq, W, 'layer_with_weights-40'), 0.30000001192092896)
    z = h @ _t(W['layer_with_weights-41/kernel']) + _t(W['layer_with_weights-41/bias'])
    return torch.softmax(z, 1).numpy()


def test_od_numpy_vs_torch():
    W = weights.synthetic(weights.OD, seed=5)
    x = np.random.default_rng(0).integers(0, 256, size=(2, 128, 151, 3)).astype(np.float32)
    a = nets.od_forward(x, W)
    b = od_torch(x, W)
    assert np.abs(a - b).max() < 1e-10


def test_keras_same_padding():
    # kernel 4 'same' pads 1 before / 2 after; stride-2 1x1 keeps even indices
    assert nets._same_pad(151, 4, 1) == (1, 2)
    assert nets._same_pad(128, 1, 2) == (0, 0)
    assert nets._same_pad(151, 2, 2) == (0, 1)
    x = np.arange(5, dtype=np.float64).reshape(1, 5, 1, 1)
    k = np.zeros((4, 1, 1, 1))
    k[0, 0, 0, 0] = 1.0      # picks x[t-1]
    y = nets.conv2d(x, k, np.zeros(1))
    assert y[0, :, 0, 0].tolist() == [0, 0, 1, 2, 3]
    mp = nets.maxpool2d_same(np.arange(1, 4, dtype=np.float64).reshape(1, 1, 3, 1))
    assert mp.ravel().tolist() == [2, 3]
