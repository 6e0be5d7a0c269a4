"""Batch-1 latency of the drop-in calls (the reference's real-time loops predict one clip per
2.56 s window): host-pointer od_pipeline / si_pipeline on 1 clip, median of 50 after warmup."""
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from mmla_audio_amd import _lib, weights  # noqa: E402
from oracle import synth  # noqa: E402

ctx = _lib.Context(0)
ctx.load_weights(weights.OD, weights.pack(weights.OD, weights.synthetic(weights.OD, seed=1)), 2)
ctx.load_weights(weights.SI, weights.pack(weights.SI, weights.synthetic(weights.SI, seed=2, n_classes=8), 8), 8,
                 _lib.HEAD_SIGMOID)
for name, fn, pcm in (('od_pipeline', ctx.od_pipeline, synth.batch(3, 1, 40960)),
                      ('si_pipeline', ctx.si_pipeline, synth.batch(4, 1, 40960)),
                      ('od_pipeline x8', ctx.od_pipeline, synth.batch(5, 8, 40960)),
                      ('od_pipeline x64', ctx.od_pipeline, synth.batch(6, 64, 40960)),
                      ('od_pipeline x256', ctx.od_pipeline, synth.batch(7, 256, 40960)),
                      ('si_pipeline x256', ctx.si_pipeline, synth.batch(8, 256, 40960))):
    for _ in range(5):
        fn(pcm)
    ts = []
    for _ in range(50):
        t = time.perf_counter()
        fn(pcm)
        ts.append(time.perf_counter() - t)
    print(f'{name:16s} median {1e3 * np.median(ts):7.3f} ms  p90 {1e3 * np.percentile(ts, 90):7.3f} ms')
