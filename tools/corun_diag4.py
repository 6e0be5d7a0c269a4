"""dev: co-run matrix.  Context a's work X on stream sa and context b's work Y on stream sb are
enqueued back to back (no host sync); each result is compared with the same work run alone.
A difference under an unrelated torch workload means a timing race inside our kernels; a
difference only next to our own kernels points at cross-context memory."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mmla_audio_amd import _lib, weights  # noqa: E402
from oracle import synth  # noqa: E402

W = weights.synthetic(weights.OD, seed=41)
N = 1024


def ctx(stream):
    c = _lib.Context(0)
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    c.set_microbatch(128, 128)
    c.set_stream(stream.cuda_stream)
    return c


def main():
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    a, b = ctx(sa), ctx(sb)
    od = torch.from_numpy(synth.batch(990, N, 40000)).cuda()
    img0 = torch.zeros((N, 128, 151, 3), dtype=torch.uint8, device='cuda')
    a.od_features_dev(od.data_ptr(), N, 40000, 40000, img=img0.data_ptr())
    mats = [torch.randn(8192, 8192, device='cuda') for _ in range(2)]
    torch.cuda.synchronize()
    out = {c: {'fe': torch.zeros_like(img0), 'net': torch.zeros((N, 2), device='cuda'),
               'pipe': torch.zeros((N, 2), device='cuda')} for c in 'ab'}

    def work(c, kind):
        o = out['a' if c is a else 'b'][kind]
        if kind == 'fe':
            c.od_features_dev(od.data_ptr(), N, 40000, 40000, img=o.data_ptr())
        elif kind == 'net':
            c.od_forward_dev(img0.data_ptr(), N, o.data_ptr(), u8=True)
        else:
            c.od_pipeline_dev(od.data_ptr(), N, 40000, 40000, o.data_ptr())

    ref = {}
    for kind in ('fe', 'net', 'pipe'):
        work(b, kind)
        torch.cuda.synchronize()
        ref[kind] = out['b'][kind].cpu().numpy().copy()
        work(a, kind)
        torch.cuda.synchronize()
        same = np.array_equal(out['a'][kind].cpu().numpy(), ref[kind])
        print(f'solo {kind}: a == b {same}', flush=True)

    def cmp(c, kind):
        g = out[c][kind].cpu().numpy()
        d = np.abs(g.astype(np.float64) - ref[kind].astype(np.float64)).reshape(N, -1).max(1)
        bad = np.nonzero(d > 0)[0]
        return f'{c}:{kind} {len(bad):3d} clips (max {d.max():.1e}, first {bad[:5].tolist()})'

    pairs = [('fe', 'net'), ('net', 'fe'), ('fe', 'pipe'), ('net', 'pipe'), ('pipe', 'net'),
             ('pipe', 'fe'), ('pipe', 'pipe'), ('mm', 'pipe'), ('mm', 'net'), ('mm', 'fe')]
    for x, y in pairs:
        for it in range(2):
            if x == 'mm':
                with torch.cuda.stream(sa):
                    for _ in range(6):
                        mats[0] @ mats[1]
            else:
                work(a, x)
            work(b, y)
            torch.cuda.synchronize()
            print(f'a {x:4s} | b {y:4s} #{it}:  ' + (cmp('a', x) + '  ' if x != 'mm' else '') + cmp('b', y),
                  flush=True)


if __name__ == '__main__':
    main()
