"""dev: find clips whose OD run trips the 3xFP16 range guard and print per-stage activation maxima"""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from mmla_audio_amd import _lib, weights
from mmla_audio_amd.synthetic import make_clips

c = _lib.Context(0)
W = weights.synthetic(weights.OD, seed=int(sys.argv[1]) if len(sys.argv) > 1 else 77)
c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
n = 32805
pcm = make_clips(n, 40000, start_index=50000)
bad = []
for c0 in range(0, n, 1024):
    m = min(1024, n - c0)
    p = torch.empty((m, 2), device='cuda')
    c.od_pipeline_dev(pcm[c0:].data_ptr(), m, 40000, 40000, p.data_ptr())
    try:
        c.range_check()
    except _lib.MmlaError:
        bad.append(c0)
print('bad chunks', bad, flush=True)
for c0 in bad[:2]:
    sub = pcm[c0:c0 + 1024].cpu().numpy()
    hits = []
    for i in range(1024):
        c.od_pipeline(sub[i:i + 1])
        if c.range_check():
            hits.append(c0 + i)
            c.release_workspace()
            c = _lib.Context(0)
            c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
        if len(hits) >= 3:
            break
    print('clips', hits, 'classes', [h % 5 for h in hits], flush=True)
    for h in hits[:2]:
        f = c.od_features(pcm[h:h + 1].cpu().numpy())
        x = f['img'].astype(np.float32)
        print('clip', h, 'img max', x.max(), 'zcr', f['zcr'].max(), flush=True)
        c.set_precision(_lib.PREC_F32)
        for st in range(12):
            t = c.debug_od_trace(x, st)
            print(f'  stage {st}: max|x| {np.abs(t).max():.4g}', flush=True)
        c.set_precision(_lib.PREC_F16X3)
