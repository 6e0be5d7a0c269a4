"""Dev tool: the OD bench sample through one build of the library.

  python tools/parity_drift.py <tag> <repo_root> [--pcm gpurun_out/drift_pcm.npy]

Runs the bench's 32-clip parity sample (first / last clip of every 16 384-clip micro-batch + 24
seeded random clips of the 65 536-clip batch, bench.sample_indices) through the library under
<repo_root>/mmla_audio_amd (the product tree or a `git worktree` of an older commit) and saves to
gpurun_out/drift_<tag>.npz: the GPU image (u8 NHWC, as the pipeline feeds the net), the
pipeline's probabilities on the sample, the net's probabilities on the GPU image (3xFP16 and exact
f32).  The first run (no --pcm) synthesises the batch and saves the sample PCM so that every build
sees the same bytes.  tools/parity_drift_report.py compares the files against the oracle on CPU.
"""
import os
import sys

import numpy as np


def main():
    tag, root = sys.argv[1], os.path.abspath(sys.argv[2])
    pcm_path = sys.argv[sys.argv.index('--pcm') + 1] if '--pcm' in sys.argv else None
    sys.path.insert(0, root)
    import torch
    from mmla_audio_amd import _lib, weights
    assert _lib.LIB_PATH.startswith(root), _lib.LIB_PATH
    os.makedirs('gpurun_out', exist_ok=True)
    if pcm_path is None:
        from mmla_audio_amd.synthetic import make_clips
        pcm = make_clips(65536, 40000)
        mb = 16384
        idx = set()
        for c0 in range(0, 65536, mb):
            idx.update((c0, c0 + mb - 1))
        idx.update(np.random.default_rng(20261015).choice(65536, 24, replace=False).tolist())
        idx = sorted(idx)
        host = pcm[idx].cpu().numpy()
        del pcm
        np.save('gpurun_out/drift_pcm.npy', host)
        np.save('gpurun_out/drift_idx.npy', np.array(idx))
    else:
        host = np.load(pcm_path)
    ctx = _lib.Context(0)
    W = weights.synthetic(weights.OD, seed=0)
    ctx.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    f = ctx.od_features(host, db=False, norm=True, zcr=True, img=True)
    probs_pipe, am, _ = ctx.od_pipeline(host)
    probs_img = ctx.od_forward(f['img'])
    ctx.set_precision(_lib.PREC_F32)
    probs_img32 = ctx.od_forward(f['img'])
    ctx.set_precision(_lib.PREC_F16X3)
    np.savez(f'gpurun_out/drift_{tag}.npz', img=f['img'], norm=f['norm'], zcr=f['zcr'],
             probs_pipe=probs_pipe, probs_img=probs_img, probs_img32=probs_img32)
    print(tag, 'ok', probs_pipe[:2].tolist(), flush=True)
    del torch


if __name__ == '__main__':
    main()
