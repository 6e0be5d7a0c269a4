"""dev: what is wrong in a front-end output computed while another context's OD-NET co-runs?
Prints, for the first corrupted clips, which frames / bands / outputs (dB, ZCR, image) differ."""
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


def ranges(idx):
    idx = sorted(set(int(i) for i in idx))
    out, s = [], None
    for i in idx:
        if s is None:
            s = e = i
        elif i == e + 1:
            e = i
        else:
            out.append((s, e))
            s = e = i
    if s is not None:
        out.append((s, e))
    return ' '.join(f'{a}' if a == b else f'{a}-{b}' for a, b in out[:12])


def main():
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    a, b = ctx(sa), ctx(sb)
    od = torch.from_numpy(synth.batch(990, N, 40000)).cuda()
    img0 = torch.zeros((N, 128, 151, 3), dtype=torch.uint8, device='cuda')
    probs = torch.zeros((N, 2), device='cuda')
    outs = {k: (torch.zeros((N, 128, 151), device='cuda'), torch.zeros((N, 151), device='cuda'),
                torch.zeros((N, 128, 151, 3), dtype=torch.uint8, device='cuda')) for k in ('ref', 'run')}

    def fe(c, k):
        db, zcr, img = outs[k]
        c.od_features_dev(od.data_ptr(), N, 40000, 40000, db=db.data_ptr(), zcr=zcr.data_ptr(),
                          img=img.data_ptr())

    a.od_features_dev(od.data_ptr(), N, 40000, 40000, img=img0.data_ptr())
    fe(a, 'ref')
    torch.cuda.synchronize()
    ref = [t.cpu().numpy() for t in outs['ref']]
    for variant in ('img+db+zcr', ):
        for it in range(6):
            fe(a, 'run')
            b.od_forward_dev(img0.data_ptr(), N, probs.data_ptr(), u8=True)
            torch.cuda.synchronize()
            got = [t.cpu().numpy() for t in outs['run']]
            bad_db = np.nonzero((got[0] != ref[0]).reshape(N, -1).any(1))[0]
            bad_z = np.nonzero((got[1] != ref[1]).any(1))[0]
            bad_i = np.nonzero((got[2] != ref[2]).reshape(N, -1).any(1))[0]
            print(f'#{it}: clips with dB diffs {len(bad_db)}, zcr diffs {len(bad_z)}, image diffs {len(bad_i)}',
                  flush=True)
            for c in bad_db[:4]:
                d = got[0][c] != ref[0][c]
                bands, frames = np.nonzero(d)
                print(f'  clip {c} (block {c % 256}, xcd-slot {c % 8}): {d.sum()} dB values differ; '
                      f'bands {ranges(bands)}; frames {ranges(frames)}; '
                      f'max |diff| {np.abs(got[0][c] - ref[0][c]).max():.3g} dB', flush=True)
            for c in bad_z[:3]:
                print(f'  clip {c}: zcr frames differ {ranges(np.nonzero(got[1][c] != ref[1][c])[0])}',
                      flush=True)
            for c in [c for c in bad_i if c not in set(bad_db)][:3]:
                d = (got[2][c] != ref[2][c])
                rows, cols, ch = np.nonzero(d)
                print(f'  clip {c}: image only: rows {ranges(rows)} cols {ranges(cols)} ch {sorted(set(ch.tolist()))}',
                      flush=True)


if __name__ == '__main__':
    main()
