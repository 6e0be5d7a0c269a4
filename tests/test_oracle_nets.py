"""CPU: the numpy net oracle against an independent torch-CPU restatement (two CPU oracles)."""
import numpy as np

from mmla_audio_amd import weights
from oracle import nets
from oracle.nets_torch import Nets


def test_od_numpy_vs_torch():
    W = weights.synthetic(weights.OD, seed=5)
    x = np.random.default_rng(0).integers(0, 256, size=(2, 128, 151, 3)).astype(np.float32)
    a = nets.od_forward(x, W)
    b = Nets(W).od_forward(x)
    assert np.abs(a - b).max() < 1e-10


def test_si_numpy_vs_torch():
    W = weights.synthetic(weights.SI, seed=6, n_classes=8)
    x = np.random.default_rng(1).normal(0, 8, size=(3, 256, 39)).astype(np.float32)
    for head in ('softmax', 'sigmoid'):
        a = nets.si_forward(x, W, head=head)
        b = Nets(W).si_forward(x, head=head)
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
