"""Diagnostic (GPU): OD pipeline results alone vs while a second context co-runs on another stream;
prints the mismatching row counts (0 and 0 = no timing-dependent kernel races)."""
import sys, numpy as np, torch
sys.path.insert(0, '.')
from mmla_audio_amd import _lib, weights
from oracle import synth
a = _lib.Context(0); b = _lib.Context(0)
W = weights.synthetic(weights.OD, seed=21)
for c in (a, b):
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
a.set_microbatch(32, 0); b.set_microbatch(32, 0)
n = 512
pcm = synth.batch(950, n, 40000)
d_pcm = torch.from_numpy(pcm).cuda()
def run(c):
    p = torch.zeros((n, 2), dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    c.od_pipeline_dev(d_pcm.data_ptr(), n, 40000, 40000, p.data_ptr(), 0)
    return p
ref = run(a); torch.cuda.synchronize(); ref = ref.cpu().numpy()
bad_solo = bad_co = 0
for it in range(6):
    p = run(a); torch.cuda.synchronize()
    bad_solo += int((p.cpu().numpy() != ref).any(1).sum())
for it in range(6):
    pa = run(a); pb = run(b)      # both contexts' streams busy at once
    torch.cuda.synchronize()
    bad_co += int((pa.cpu().numpy() != ref).any(1).sum()) + int((pb.cpu().numpy() != ref).any(1).sum())
print('solo mismatching rows', bad_solo, 'co-run mismatching rows', bad_co, flush=True)
