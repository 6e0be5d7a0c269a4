"""Timing independence: the OD and SI pipelines give bit-identical results whether they run alone
or while a second context's kernels co-run on another stream (a kernel with a missing barrier or
an unordered LDS/global dependency would drift under the changed co-residency)."""
import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu


def _ctx(seed):
    from mmla_audio_amd import _lib, weights
    c = _lib.Context(0)
    c.load_weights(weights.OD, weights.pack(weights.OD, weights.synthetic(weights.OD, seed=seed)), 2)
    Ws = weights.synthetic(weights.SI, seed=seed + 1, n_classes=8)
    c.load_weights(weights.SI, weights.pack(weights.SI, Ws, 8), 8, 1)
    c.set_microbatch(64, 64)
    return c


def test_corun_bit_identical():
    import torch
    a, b = _ctx(41), _ctx(41)
    n = 256
    od = torch.from_numpy(synth.batch(990, n, 40000)).cuda()
    si = torch.from_numpy(synth.batch(991, n, 24000)).cuda()

    def run(c):
        po = torch.zeros((n, 2), dtype=torch.float32, device='cuda')
        ps = torch.zeros((n, 8), dtype=torch.float32, device='cuda')
        torch.cuda.synchronize()
        c.od_pipeline_dev(od.data_ptr(), n, 40000, 40000, po.data_ptr(), 0)
        c.si_pipeline_dev(si.data_ptr(), n, 24000, 24000, ps.data_ptr(), 0)
        return po, ps

    ro, rs = run(a)
    torch.cuda.synchronize()
    ro, rs = ro.cpu().numpy(), rs.cpu().numpy()
    for _ in range(3):
        (ao, as_), (bo, bs) = run(a), run(b)   # both contexts' streams busy at once
        torch.cuda.synchronize()
        for o, s_ in ((ao, as_), (bo, bs)):
            assert np.array_equal(o.cpu().numpy(), ro)
            assert np.array_equal(s_.cpu().numpy(), rs)
