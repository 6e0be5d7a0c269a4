"""Dev: batch-1 OD host-pointer calls only (for a rocprof kernel-trace of the latency path)."""
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from mmla_audio_amd import _lib, weights  # noqa: E402
from oracle import synth  # noqa: E402

ctx = _lib.Context(0)
ctx.load_weights(weights.OD, weights.pack(weights.OD, weights.synthetic(weights.OD, seed=1)), 2)
pcm = synth.batch(3, 1, 40960)
for _ in range(5):
    ctx.od_pipeline(pcm)
ts = []
for _ in range(100):
    t = time.perf_counter()
    ctx.od_pipeline(pcm)
    ts.append(time.perf_counter() - t)
print(f'od batch-1 median {1e3 * np.median(ts):.3f} ms over 100 calls')
