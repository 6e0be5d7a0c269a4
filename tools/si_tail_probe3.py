"""dev: SI 65 536 clips with a forced micro-batch vs 4096-clip chunks"""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from mmla_audio_amd import _lib, weights
from mmla_audio_amd.synthetic import make_clips

c = _lib.Context(0)
W = weights.synthetic(weights.SI, seed=78, n_classes=630)
c.load_weights(weights.SI, weights.pack(weights.SI, W, 630), 630, _lib.HEAD_SOFTMAX)
n = 65536
pcm = make_clips(n, 24000, start_index=70000)
pb = torch.empty((n, 630), device='cuda')
for c0 in range(0, n, 4096):
    c.si_pipeline_dev(pcm[c0:].data_ptr(), 4096, 24000, 24000, pb[c0:].data_ptr())
c.synchronize()
for mb in (61440, 40000, 65536):
    c.set_microbatch(0, mb)
    probs = torch.empty((n, 630), device='cuda')
    c.si_pipeline_dev(pcm.data_ptr(), n, 24000, 24000, probs.data_ptr())
    c.synchronize()
    d = (probs != pb).any(1).nonzero().flatten()
    print('mb', mb, 'rows differing', d.numel(), d[:5].tolist(), d[-5:].tolist() if d.numel() else [], flush=True)
c.set_microbatch(0, 0)
print('auto mb', c.get_microbatch())
