"""Dev tool: compare tools/parity_drift.py outputs against the oracle (CPU).

  python tools/parity_drift_report.py tagA tagB ...

For each build: pixels differing from the oracle image (and from the first build's image), the
log-probability error of the pipeline against the oracle net on the ORACLE image (the bench's old
figure, which mixes image LSBs and net arithmetic), the net's error on the GPU's OWN image (3xFP16
and f32), and per clip which clips carry the error.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mmla_audio_amd import weights  # noqa: E402
from oracle import compare, od_fe  # noqa: E402
from oracle.nets_torch import Nets  # noqa: E402


def per_clip_logp(p, ref):
    with np.errstate(divide='ignore'):
        return np.abs(np.log(p.astype(np.float64)) - np.log(ref)).max(1)


def main():
    tags = sys.argv[1:]
    pcm = np.load(os.path.join(REPO, 'gpurun_out/drift_pcm.npy'))
    idx = np.load(os.path.join(REPO, 'gpurun_out/drift_idx.npy'))
    feats = [od_fe.od_features(pcm[j]) for j in range(len(pcm))]
    oimg = np.stack([f['png_rgb'] for f in feats])
    net = Nets(weights.synthetic(weights.OD, seed=0))
    ref_oimg = net.od_forward(oimg.astype(np.float32))
    first = None
    for t in tags:
        d = np.load(os.path.join(REPO, f'gpurun_out/drift_{t}.npz'))
        img = d['img']
        ref_gimg = net.od_forward(img.astype(np.float32))
        lsb = np.abs(img.astype(int) - oimg.astype(int))
        print(f'== {t}')
        print(f'  image vs oracle: {int((lsb > 0).sum())} pixel values off (max {lsb.max()} LSB) of {lsb.size}; '
              f'clips with any: {int((lsb.reshape(len(img), -1).max(1) > 0).sum())}')
        if first is not None:
            dd = np.abs(img.astype(int) - first.astype(int))
            print(f'  image vs {tags[0]}: {int((dd > 0).sum())} pixel values differ')
        else:
            first = img
        print(f'  pipeline vs oracle net on oracle image: logp {compare.logp_err(d["probs_pipe"], ref_oimg):.3g}')
        print(f'  pipeline vs oracle net on GPU image:    logp {compare.logp_err(d["probs_pipe"], ref_gimg):.3g}')
        print(f'  net(GPU image) 3xFP16 vs oracle same image: logp {compare.logp_err(d["probs_img"], ref_gimg):.3g}')
        print(f'  net(GPU image) f32    vs oracle same image: logp {compare.logp_err(d["probs_img32"], ref_gimg):.3g}')
        print(f'  pipeline == net(GPU image) bitwise: {np.array_equal(d["probs_pipe"], d["probs_img"])}')
        e_o = per_clip_logp(d['probs_pipe'], ref_oimg)
        e_g = per_clip_logp(d['probs_pipe'], ref_gimg)
        npx = (lsb.reshape(len(img), -1) > 0).sum(1)
        worst = np.argsort(-e_o)[:6]
        for j in worst:
            print(f'    clip {idx[j]:6d} (class {idx[j] % 5}): logp err vs oracle-image net {e_o[j]:.3g}, '
                  f'vs own-image net {e_g[j]:.3g}, {npx[j]} LSB pixels, p={d["probs_pipe"][j].tolist()}')


if __name__ == '__main__':
    main()
