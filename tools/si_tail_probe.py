"""dev: where does a 65 536-clip SI run diverge from the same clips run in 4096-clip batches?"""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from mmla_audio_amd import _lib, weights
from mmla_audio_amd.synthetic import make_clips

c = _lib.Context(0)
W = weights.synthetic(weights.SI, seed=78, n_classes=630)
c.load_weights(weights.SI, weights.pack(weights.SI, W, 630), 630, _lib.HEAD_SOFTMAX)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
pcm = make_clips(n, 24000, start_index=70000)
feat = torch.empty((n, 256, 39), device='cuda')
c.si_features_dev(pcm.data_ptr(), n, 24000, 24000, feat.data_ptr())
probs = torch.empty((n, 630), device='cuda')
c.si_pipeline_dev(pcm.data_ptr(), n, 24000, 24000, probs.data_ptr())
c.synchronize()
fb = torch.empty_like(feat)
pb = torch.empty_like(probs)
for c0 in range(0, n, 4096):
    m = min(4096, n - c0)
    c.si_features_dev(pcm[c0:].data_ptr(), m, 24000, 24000, fb[c0:].data_ptr())
    c.si_pipeline_dev(pcm[c0:].data_ptr(), m, 24000, 24000, pb[c0:].data_ptr())
c.synchronize()
df = (feat != fb).flatten(1).any(1).nonzero().flatten()
dp = (probs != pb).any(1).nonzero().flatten()
print('feature rows differing', df.numel(), df[:5].tolist(), df[-5:].tolist() if df.numel() else [])
print('prob rows differing', dp.numel(), dp[:5].tolist(), dp[-5:].tolist() if dp.numel() else [])
# the f32 path on the same batch
c.set_precision(_lib.PREC_F32)
p32 = torch.empty_like(probs)
c.si_pipeline_dev(pcm.data_ptr(), n, 24000, 24000, p32.data_ptr())
c.synchronize()
pb32 = torch.empty_like(probs)
for c0 in range(0, n, 4096):
    m = min(4096, n - c0)
    c.si_pipeline_dev(pcm[c0:].data_ptr(), m, 24000, 24000, pb32[c0:].data_ptr())
c.synchronize()
d32 = (p32 != pb32).any(1).nonzero().flatten()
print('f32 prob rows differing', d32.numel(), d32[:5].tolist(), d32[-5:].tolist() if d32.numel() else [])
