"""dev: localise a co-run / fresh-context difference of the OD pipeline (tests/test_gpu_corun.py).

Prints, per scenario, how many clips' probabilities differ from context a's solo run and by how
much: a again (determinism), a fresh context b run alone, then a and b co-running on two streams;
the same for the front-end image alone and for OD-NET alone on a fixed image.  Run it with and
without MMLA_WS_POISON=0xff (new workspace slots filled with NaN bytes)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mmla_audio_amd import _lib, weights  # noqa: E402
from oracle import synth  # noqa: E402


def ctx(stream):
    c = _lib.Context(0)
    c.load_weights(weights.OD, weights.pack(weights.OD, weights.synthetic(weights.OD, seed=41)), 2)
    c.set_microbatch(128, 128)
    c.set_stream(stream.cuda_stream)
    return c


def report(tag, got, ref):
    g, r = got.cpu().numpy(), ref
    d = np.abs(g.astype(np.float64) - r.astype(np.float64)).reshape(len(r), -1)
    bad = np.nonzero(d.max(1) > 0)[0]
    nan = int(np.isnan(g).any(axis=tuple(range(1, g.ndim))).sum())
    print(f'{tag:28s} clips differing {len(bad):5d}  max {np.nanmax(d) if d.size else 0:.3e}  '
          f'nan clips {nan}  first {bad[:16].tolist()}', flush=True)


def main():
    n = 1024
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    a = ctx(sa)
    od = torch.from_numpy(synth.batch(990, n, 40000)).cuda()
    P = {k: torch.zeros((n, 2), device='cuda') for k in ('solo', 'a', 'b')}
    I = {k: torch.zeros((n, 128, 151, 3), dtype=torch.uint8, device='cuda') for k in ('solo', 'a', 'b')}
    F = {k: torch.zeros((n, 2), device='cuda') for k in ('solo', 'a', 'b')}
    torch.cuda.synchronize()

    def pipe(c, k):
        c.od_pipeline_dev(od.data_ptr(), n, 40000, 40000, P[k].data_ptr())

    def fe(c, k):
        c.od_features_dev(od.data_ptr(), n, 40000, 40000, img=I[k].data_ptr())

    def net(c, k):
        c.od_forward_dev(I['solo'].data_ptr(), n, F[k].data_ptr(), u8=True)

    for name, fn, out in (('pipeline', pipe, P), ('front-end', fe, I), ('net', net, F)):
        fn(a, 'solo')
        torch.cuda.synchronize()
        ref = out['solo'].cpu().numpy()
        fn(a, 'a')
        torch.cuda.synchronize()
        report(f'{name}: a again', out['a'], ref)
        b = ctx(sb)
        fn(b, 'b')
        torch.cuda.synchronize()
        report(f'{name}: fresh b alone', out['b'], ref)
        fn(b, 'b')
        torch.cuda.synchronize()
        report(f'{name}: b again', out['b'], ref)
        for it in range(3):
            fn(a, 'a')
            fn(b, 'b')
            torch.cuda.synchronize()
            report(f'{name}: co-run {it} a', out['a'], ref)
            report(f'{name}: co-run {it} b', out['b'], ref)
        b.close() if hasattr(b, 'close') else None
        del b


if __name__ == '__main__':
    main()
