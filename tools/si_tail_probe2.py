"""dev: SI host-mode vs device-mode results on a sample of a 65 536-clip batch"""
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
probs = torch.empty((n, 630), device='cuda')
c.si_pipeline_dev(pcm.data_ptr(), n, 24000, 24000, probs.data_ptr())
c.synchronize()
idx = sorted(set([0, 65535, 32767, 32768] + np.random.default_rng(2).choice(n, 32, replace=False).tolist()))
sub_d = pcm[idx].contiguous()
sub = sub_d.cpu().numpy()
pd = torch.empty((len(idx), 630), device='cuda')
c.si_pipeline_dev(sub_d.data_ptr(), len(idx), 24000, 24000, pd.data_ptr())
c.synchronize()
ph, _, _ = c.si_pipeline(sub)
big = probs[idx].cpu().numpy()
pd = pd.cpu().numpy()
for j, i in enumerate(idx):
    one, _, _ = c.si_pipeline(sub[j:j + 1])
    print(i, (70000 + i) % 5, 'zero' if not sub[j].any() else 'nz', 'big==dev_sub', np.array_equal(big[j], pd[j]),
          'host==dev_sub', np.array_equal(ph[j], pd[j]), 'one==host', np.array_equal(one[0], ph[j]),
          'big==one', np.array_equal(big[j], one[0]))
