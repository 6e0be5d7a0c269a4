"""dev: replay the range-guard tests, then diff a 65 536-clip SI run against 4096-clip chunks"""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import test_gpu_range_guard as rg
from mmla_audio_amd import _lib, weights
from mmla_audio_amd.synthetic import make_clips

which = sys.argv[1:] or ['all']
for name in dir(rg):
    if name.startswith('test_') and ('all' in which or name in which):
        getattr(rg, name)()
        print('ran', name, flush=True)
import test_gpu_fullsize as fs
if 'od' in sys.argv[1:] or 'all' in which:
    fs.test_od_two_microbatches('f16x3')
    fs.test_od_two_microbatches('f32')
    print('ran od fullsize', flush=True)
c = _lib.Context(0)
W = weights.synthetic(weights.SI, seed=78, n_classes=630)
c.load_weights(weights.SI, weights.pack(weights.SI, W, 630), 630, _lib.HEAD_SOFTMAX)
n = 65536
print('mb', c.get_microbatch(), flush=True)
pcm = make_clips(n, 24000, start_index=70000)
feat = torch.empty((n, 256, 39), device='cuda')
c.si_features_dev(pcm.data_ptr(), n, 24000, 24000, feat.data_ptr())
probs = torch.empty((n, 630), device='cuda')
c.si_pipeline_dev(pcm.data_ptr(), n, 24000, 24000, probs.data_ptr())
c.synchronize()
print('reruns', c.range_check(), flush=True)
fb = torch.empty_like(feat)
pb = torch.empty_like(probs)
for c0 in range(0, n, 4096):
    c.si_features_dev(pcm[c0:].data_ptr(), 4096, 24000, 24000, fb[c0:].data_ptr())
    c.si_pipeline_dev(pcm[c0:].data_ptr(), 4096, 24000, 24000, pb[c0:].data_ptr())
c.synchronize()
df = (feat != fb).flatten(1).any(1).nonzero().flatten()
dp = (probs != pb).any(1).nonzero().flatten()
print('feature rows differing', df.numel(), df[:5].tolist(), df[-5:].tolist() if df.numel() else [])
print('prob rows differing', dp.numel(), dp[:8].tolist(), dp[-8:].tolist() if dp.numel() else [])
idx = sorted(set([0, 65535, 32767, 32768] + np.random.default_rng(2).choice(n, 32, replace=False).tolist()))
c.release_workspace()
p1, _, _ = c.si_pipeline(pcm[idx].cpu().numpy())
dh = [i for j, i in enumerate(idx) if not np.array_equal(p1[j], probs[i].cpu().numpy())]
print('host small-batch rows differing from big', dh)
if dp.numel():
    z = torch.zeros((1, 24000), dtype=torch.int16, device='cuda')
    pz = torch.empty((1, 630), device='cuda')
    c.si_pipeline_dev(z.data_ptr(), 1, 24000, 24000, pz.data_ptr())
    c.synchronize()
    bad = dp[:8]
    print('bad rows == zero-clip output', [(int(i), bool(torch.equal(probs[i], pz[0]))) for i in bad])
    print('bad rows chunk == zero-clip', [(int(i), bool(torch.equal(pb[i], pz[0]))) for i in bad])
    print('first bad block of 256', int(dp.min()) // 256, 'count', dp.numel())
