"""Stream ordering of one context's workspaces (include/mmla.h mmla_set_stream).

A device-pointer call only enqueues; switching the context to another stream while that work is
in flight must not let the next call reuse its workspaces early (mmla_set_stream makes the new
stream wait for the old one).  Results must equal the serial run bit for bit.
"""
import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu


def _od_ctx():
    from mmla_audio_amd import _lib, weights
    c = _lib.Context(0)
    c.load_weights(weights.OD, weights.pack(weights.OD, weights.synthetic(weights.OD, seed=44)), 2)
    return c


def test_switch_stream_between_async_calls():
    import torch
    n = 1024
    c = _od_ctx()
    c.set_microbatch(256, 0)   # several micro-batches: the second call's image slot is live early
    x1 = torch.from_numpy(synth.batch(1200, n, 40000)).cuda()
    x2 = torch.from_numpy(synth.batch(1300, n, 40000)).cuda()

    def run_serial(x):
        p = torch.zeros((n, 2), dtype=torch.float32, device='cuda')
        torch.cuda.synchronize()
        c.set_stream(None)
        c.od_pipeline_dev(x.data_ptr(), n, 40000, 40000, p.data_ptr())
        c.synchronize()
        return p.cpu().numpy()

    r1, r2 = run_serial(x1), run_serial(x2)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    p1 = torch.zeros((n, 2), dtype=torch.float32, device='cuda')
    p2 = torch.zeros((n, 2), dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    c.set_stream(sa.cuda_stream)
    c.od_pipeline_dev(x1.data_ptr(), n, 40000, 40000, p1.data_ptr())
    c.set_stream(sb.cuda_stream)          # no host sync in between
    c.od_pipeline_dev(x2.data_ptr(), n, 40000, 40000, p2.data_ptr())
    torch.cuda.synchronize()
    c.set_stream(None)
    assert np.array_equal(p1.cpu().numpy(), r1)
    assert np.array_equal(p2.cpu().numpy(), r2)
