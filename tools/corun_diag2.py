"""dev: bisect the co-run difference of context b's OD pipeline (tools/corun_diag.py found it):
context b runs the pipeline on stream sb while context a runs <other> on stream sa, enqueued first
with no host sync in between; b's probabilities are compared with b's solo run."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mmla_audio_amd import _lib, weights  # noqa: E402
from oracle import synth  # noqa: E402


def ctx(stream, prec=None):
    c = _lib.Context(0)
    c.load_weights(weights.OD, weights.pack(weights.OD, weights.synthetic(weights.OD, seed=41)), 2)
    c.set_microbatch(128, 128)
    if prec is not None:
        c.set_precision(prec)
    c.set_stream(stream.cuda_stream)
    return c


def diff(got, ref):
    d = np.abs(got.cpu().numpy().astype(np.float64) - ref.astype(np.float64)).reshape(len(ref), -1)
    bad = np.nonzero(d.max(1) > 0)[0]
    return f'clips differing {len(bad):4d} max {d.max():.2e} first {bad[:8].tolist()}'


def main():
    n = 1024
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    od = torch.from_numpy(synth.batch(990, n, 40000)).cuda()
    img = torch.zeros((n, 128, 151, 3), dtype=torch.uint8, device='cuda')
    pa = torch.zeros((n, 2), device='cuda')
    pb = torch.zeros((n, 2), device='cuda')
    ia = torch.zeros((n, 128, 151, 3), dtype=torch.uint8, device='cuda')
    for prec_name, prec in (('f16x3', None), ('f32', _lib.PREC_F32)):
        a, b = ctx(sa, prec), ctx(sb, prec)
        a.od_features_dev(od.data_ptr(), n, 40000, 40000, img=img.data_ptr())
        b.od_pipeline_dev(od.data_ptr(), n, 40000, 40000, pb.data_ptr())
        a.od_pipeline_dev(od.data_ptr(), n, 40000, 40000, pa.data_ptr())
        torch.cuda.synchronize()
        ref = pb.cpu().numpy()
        print(f'[{prec_name}] a solo pipeline vs b solo pipeline: {diff(pa, ref)}', flush=True)
        others = {
            'pipeline': lambda: a.od_pipeline_dev(od.data_ptr(), n, 40000, 40000, pa.data_ptr()),
            'front-end': lambda: a.od_features_dev(od.data_ptr(), n, 40000, 40000, img=ia.data_ptr()),
            'net': lambda: a.od_forward_dev(img.data_ptr(), n, pa.data_ptr(), u8=True),
        }
        for name, other in others.items():
            for it in range(2):
                other()
                b.od_pipeline_dev(od.data_ptr(), n, 40000, 40000, pb.data_ptr())
                torch.cuda.synchronize()
                print(f'[{prec_name}] b pipeline while a runs {name:10s} #{it}: {diff(pb, ref)}', flush=True)
        # b's pipeline first, a's second: does the later-enqueued context always drift?
        b.od_pipeline_dev(od.data_ptr(), n, 40000, 40000, pb.data_ptr())
        a.od_pipeline_dev(od.data_ptr(), n, 40000, 40000, pa.data_ptr())
        torch.cuda.synchronize()
        print(f'[{prec_name}] b enqueued first: b {diff(pb, ref)} | a {diff(pa, ref)}', flush=True)
        a.close()
        b.close()


if __name__ == '__main__':
    main()
