"""dev: which co-running kernel corrupts the OD front-end?  Context a enqueues K front-end calls
(distinct dB outputs) on its stream; context b then runs one candidate workload on its own stream;
every front-end output is compared with a solo run."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mmla_audio_amd import _lib, weights  # noqa: E402

if os.environ.get('MMLA_LIB'):
    _lib.load_library(os.environ['MMLA_LIB'])
from oracle import synth  # noqa: E402

W = weights.synthetic(weights.OD, seed=41)
N, K = 4096, 12


def ctx(stream, prec=None):
    c = _lib.Context(0)
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    c.set_microbatch(512, 128)
    if prec is not None:
        c.set_precision(prec)
    c.set_stream(stream.cuda_stream)
    return c


def main():
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    a = ctx(sa)
    b16, b32 = ctx(sb), ctx(sb, _lib.PREC_F32)
    od = torch.from_numpy(synth.batch(990, N, 40000)).cuda()
    img0 = torch.zeros((N, 128, 151, 3), dtype=torch.uint8, device='cuda')
    dbs = [torch.zeros((N, 128, 151), device='cuda') for _ in range(K)]
    probs = torch.zeros((N, 2), device='cuda')
    a.od_features_dev(od.data_ptr(), N, 40000, 40000, db=dbs[0].data_ptr(), img=img0.data_ptr())
    torch.cuda.synchronize()
    ref = dbs[0].cpu().numpy()
    x = img0[:256].cpu().numpy().astype(np.float32)
    cands = {
        'nothing': lambda: None,
        'net f16x3': lambda: b16.od_forward_dev(img0.data_ptr(), N, probs.data_ptr(), u8=True),
        'net f32': lambda: b32.od_forward_dev(img0.data_ptr(), N, probs.data_ptr(), u8=True),
        'trace 1 (stem+blk1 resblk)': lambda: b16.debug_od_trace(x, 1),
        'trace 3 (blocks 1-3 resblk)': lambda: b16.debug_od_trace(x, 3),
        'trace 9 (+conv_h3 4-9)': lambda: b16.debug_od_trace(x, 9),
    }
    for name, fn in cands.items():
        for it in range(2):
            for d in dbs:
                a.od_features_dev(od.data_ptr(), N, 40000, 40000, db=d.data_ptr())
            fn()
            torch.cuda.synchronize()
            nbad = [int((d.cpu().numpy() != ref).reshape(N, -1).any(1).sum()) for d in dbs]
            print(f'{name:30s} #{it}: corrupted clips per front-end call {nbad}', flush=True)


if __name__ == '__main__':
    main()
