"""Timing independence: the OD and SI pipelines give bit-identical results whether they run alone
or while a second context's kernels co-run on another stream (a kernel with a missing barrier or
an unordered LDS/global dependency would drift under the changed co-residency).

Both contexts' work is enqueued back to back with no host synchronisation in between; events on the
two streams show that context b's first kernel was eligible to start before context a finished.
"""
import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu


def _ctx(seed, stream):
    from mmla_audio_amd import _lib, weights
    c = _lib.Context(0)
    c.load_weights(weights.OD, weights.pack(weights.OD, weights.synthetic(weights.OD, seed=seed)), 2)
    Ws = weights.synthetic(weights.SI, seed=seed + 1, n_classes=8)
    c.load_weights(weights.SI, weights.pack(weights.SI, Ws, 8), 8, 1)
    c.set_microbatch(128, 128)
    c.set_stream(stream.cuda_stream)
    return c


def test_corun_bit_identical():
    import torch
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    a, b = _ctx(41, sa), _ctx(41, sb)
    n = 1024
    od = torch.from_numpy(synth.batch(990, n, 40000)).cuda()
    si = torch.from_numpy(synth.batch(991, n, 24000)).cuda()
    outs = {k: (torch.zeros((n, 2), device='cuda'), torch.zeros((n, 8), device='cuda'))
            for k in ('solo', 'a', 'b')}

    def enqueue(c, po, ps):
        c.od_pipeline_dev(od.data_ptr(), n, 40000, 40000, po.data_ptr())
        c.si_pipeline_dev(si.data_ptr(), n, 24000, 24000, ps.data_ptr())

    torch.cuda.synchronize()
    enqueue(a, *outs['solo'])
    torch.cuda.synchronize()
    ro, rs = (t.cpu().numpy() for t in outs['solo'])
    for _ in range(3):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record(sa)
        enqueue(a, *outs['a'])
        ev[1].record(sa)
        ev[2].record(sb)
        enqueue(b, *outs['b'])        # no synchronisation between the two contexts
        ev[3].record(sb)
        torch.cuda.synchronize()
        a_end = ev[0].elapsed_time(ev[1])
        b_start = ev[0].elapsed_time(ev[2])
        assert b_start < a_end, f'b eligible at {b_start:.2f} ms, a ran until {a_end:.2f} ms'
        for k in ('a', 'b'):
            assert np.array_equal(outs[k][0].cpu().numpy(), ro)
            assert np.array_equal(outs[k][1].cpu().numpy(), rs)
