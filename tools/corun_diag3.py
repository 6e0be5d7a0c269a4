"""dev: which OD pipeline result is right?  Fresh contexts with different histories and micro-batch
sizes against the composed result net(front-end(all clips)) and the float64 oracle on a few clips."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mmla_audio_amd import _lib, weights  # noqa: E402
from oracle import nets, od_fe, synth  # noqa: E402

W = weights.synthetic(weights.OD, seed=41)


STREAMS = []


def ctx(mb):
    c = _lib.Context(0)
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    c.set_microbatch(mb, 128)
    if os.environ.get('DIAG_STREAM') == 'torch':
        STREAMS.append(torch.cuda.Stream())
        c.set_stream(STREAMS[-1].cuda_stream)
    return c


def diff(got, ref):
    d = np.abs(got.astype(np.float64) - ref.astype(np.float64)).reshape(len(ref), -1)
    bad = np.nonzero(d.max(1) > 0)[0]
    return f'differing {len(bad):4d} max {d.max():.2e} first {bad[:8].tolist()}'


def main():
    n = 1024
    pcm = synth.batch(990, n, 40000)
    od = torch.from_numpy(pcm).cuda()
    img = torch.zeros((n, 128, 151, 3), dtype=torch.uint8, device='cuda')
    p = torch.zeros((n, 2), device='cuda')

    def pipe(c):
        c.od_pipeline_dev(od.data_ptr(), n, 40000, 40000, p.data_ptr())
        torch.cuda.synchronize()
        return p.cpu().numpy().copy()

    c = ctx(128)
    c.od_features_dev(od.data_ptr(), n, 40000, 40000, img=img.data_ptr())
    c.od_forward_dev(img.data_ptr(), n, p.data_ptr(), u8=True)
    torch.cuda.synchronize()
    comp = p.cpu().numpy().copy()
    imgs = img.cpu().numpy()
    c.close()
    idx = [0, 1, 127, 128, 130, 131, 155, 181, 255, 256, 1023]
    ref = np.array([nets.od_forward(imgs[i:i + 1].astype(np.float32), W)[0] for i in idx])
    print('composed vs oracle on', idx, diff(comp[idx], ref), flush=True)
    fe_ref = od_fe.od_features(pcm[130])
    print('front-end image clip 130 vs oracle: max |diff|',
          np.abs(imgs[130].astype(int) - fe_ref['png_rgb'].astype(int)).max(), flush=True)
    for name, mb, hist in (('pipeline mb 128 fresh', 128, False), ('pipeline mb 128 again', 128, None),
                           ('pipeline mb 1024 fresh', 1024, False),
                           ('pipeline mb 128 after FE-only', 128, True),
                           ('pipeline mb 256 fresh', 256, False)):
        if hist is not None:
            c = ctx(mb)
            if hist:
                c.od_features_dev(od.data_ptr(), n, 40000, 40000, img=img.data_ptr())
        got = pipe(c)
        print(f'{name:32s} vs composed: {diff(got, comp)} | oracle clips: {diff(got[idx], ref)}',
              flush=True)


if __name__ == '__main__':
    main()
