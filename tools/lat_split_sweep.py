"""Dev: host-pointer od_pipeline / si_pipeline latency over batch sizes around the BiLSTM split
threshold (run with MMLA_LSTM_SPLIT_MAX=0 and =256 to compare the two BiLSTM kernels)."""
import os
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
print('MMLA_LSTM_SPLIT_MAX =', os.environ.get('MMLA_LSTM_SPLIT_MAX'))
for n in (32, 64, 96, 128, 192, 256):
    row = []
    for fn, seed in ((ctx.od_pipeline, 10), (ctx.si_pipeline, 11)):
        pcm = synth.batch(seed + n, n, 40960)
        for _ in range(3):
            fn(pcm)
        ts = []
        for _ in range(20):
            t = time.perf_counter()
            fn(pcm)
            ts.append(time.perf_counter() - t)
        row.append(1e3 * np.median(ts))
    print(f'n={n:4d}  od {row[0]:7.3f} ms  si {row[1]:7.3f} ms')
