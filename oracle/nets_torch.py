"""torch-CPU restatement of the two Keras graphs -- TEST INFRASTRUCTURE ONLY.

An independent second CPU oracle for ``oracle/nets.py`` (tests/test_oracle_nets.py checks them
against each other at 1e-10 in float64), and the batched, all-core network leg of bench.py's
best-effort CPU baseline (SURVEY.md 8(d) mode ii) in float32.  Same graphs and citations as
``oracle/nets.py``: OD ``overlap_detector_temp.py:253-303``, SI ``speaker_identification.py:
168-218,401-410``; Keras 'same' padding, BN eps 1e-3, LSTM gates i,f,c,o (torch's i,f,g,o order is
the same), Bidirectional concat of [h_fwd(T-1), h_bwd(after x[0])].
"""
import numpy as np
import torch
import torch.nn.functional as F

POOL = (True, False, False, True, False, False, True, False, False)
LEAKY_ALPHA = 0.30000001192092896   # float32(0.3)


class Nets:
    """OD / SI forward over a weight dict (variables.index names), tensors cached per dtype."""

    def __init__(self, W, dtype=torch.float64):
        self.dtype = dtype
        self.W = {k: torch.as_tensor(np.asarray(v, np.float64)).to(dtype) for k, v in W.items()}
        self._lstm = {}

    def _w(self, k, var):
        return self.W[f'layer_with_weights-{k}/{var}']

    @staticmethod
    def _pads(n, kk, s):
        out = -(-n // s)
        tot = max((out - 1) * s + kk - n, 0)
        return tot // 2, tot - tot // 2

    def conv2d(self, x, k, stride=1):
        """x NCHW; kernel [kh, kw, cin, cout] (Keras) with 'same' padding."""
        ker = self._w(k, 'kernel')
        kh, kw = ker.shape[:2]
        ph, pw = self._pads(x.shape[2], kh, stride), self._pads(x.shape[3], kw, stride)
        xp = F.pad(x, (pw[0], pw[1], ph[0], ph[1]))
        return F.conv2d(xp, ker.permute(3, 2, 0, 1), self._w(k, 'bias'), stride=stride)

    def conv1d(self, x, k, stride=1):
        """x NCT; kernel [k, cin, cout]."""
        ker = self._w(k, 'kernel')
        p = self._pads(x.shape[2], ker.shape[0], stride)
        return F.conv1d(F.pad(x, p), ker.permute(2, 1, 0), self._w(k, 'bias'), stride=stride)

    def bn(self, x, k):
        return F.batch_norm(x, self._w(k, 'moving_mean'), self._w(k, 'moving_variance'),
                            self._w(k, 'gamma'), self._w(k, 'beta'), False, 0.0, 1e-3)

    def bilstm(self, seq, k):
        if k not in self._lstm:
            p = f'layer_with_weights-{k}'
            m = torch.nn.LSTM(seq.shape[-1], 256, batch_first=True, bidirectional=True).to(self.dtype)
            with torch.no_grad():
                for side, suf in (('forward', ''), ('backward', '_reverse')):
                    getattr(m, 'weight_ih_l0' + suf).copy_(self.W[f'{p}/{side}/kernel'].T)
                    getattr(m, 'weight_hh_l0' + suf).copy_(self.W[f'{p}/{side}/recurrent_kernel'].T)
                    getattr(m, 'bias_ih_l0' + suf).copy_(self.W[f'{p}/{side}/bias'])
                    getattr(m, 'bias_hh_l0' + suf).zero_()
            self._lstm[k] = m
        out, _ = self._lstm[k](seq)
        return torch.cat([out[:, -1, :256], out[:, 0, 256:]], dim=1)

    @torch.no_grad()
    def od_forward(self, x):
        """x [N,128,151,3] PNG values -> softmax probs [N,2] (numpy)."""
        x = torch.as_tensor(np.asarray(x)).to(self.dtype).permute(0, 3, 1, 2)
        net = self.conv2d(x, 0)
        k = 1
        for pool in POOL:
            out = self.conv2d(F.elu(self.bn(net, k)), k + 1)
            out = self.conv2d(F.elu(self.bn(out, k + 2)), k + 3)
            if pool:
                res = self.conv2d(net, k + 4, 2)
                h, w = out.shape[2], out.shape[3]
                out = F.max_pool2d(F.pad(out, (0, w % 2, 0, h % 2), value=-np.inf), 2)
                k += 5
            else:
                res = net
                k += 4
            net = res + out
        seq = net.mean(dim=2).permute(0, 2, 1)
        h = F.leaky_relu(self.bilstm(seq, 40), LEAKY_ALPHA)
        z = h @ self.W['layer_with_weights-41/kernel'] + self.W['layer_with_weights-41/bias']
        return torch.softmax(z, 1).numpy()

    @torch.no_grad()
    def si_forward(self, x, head='softmax'):
        """x [N,256,39] -> [N,K] (softmax base model or sigmoid deployed head)."""
        x = torch.as_tensor(np.asarray(x)).to(self.dtype).permute(0, 2, 1)
        net = self.conv1d(x, 0)
        k = 1
        for pool in POOL:
            inp = net
            if pool:
                t = net.shape[2]
                inp = F.max_pool1d(F.pad(net, (0, t % 2), value=-np.inf), 2)
            out = self.conv1d(F.relu(self.bn(inp, k)), k + 1)
            out = F.relu(self.bn(out, k + 2))
            if pool:
                res = self.conv1d(net, k + 3, 2)
                out = self.conv1d(out, k + 4)
                k += 5
            else:
                res = net
                out = self.conv1d(out, k + 3)
                k += 4
            net = res + out
        net = F.relu(self.bn(net, 40))
        t = net.shape[2] // 4 * 4
        net = F.avg_pool1d(net[:, :, :t], 4)
        h = self.bilstm(net.permute(0, 2, 1), 41)
        z = h @ self.W['layer_with_weights-42/kernel'] + self.W['layer_with_weights-42/bias']
        return (torch.softmax(z, 1) if head == 'softmax' else torch.sigmoid(z)).numpy()
