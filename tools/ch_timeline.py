"""Phase timeline of conv_h3 launches (dev tool): needs a library built with -DCH_EXP=1
(make -C mmla_audio_amd/csrc variant VSRC=conv_h3 VDEF=-DCH_EXP=1 VNAME=chexp).  Runs the OD
pipeline on 4096 clips once per selected layer and prints the median phase cycles per wave."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, '.')
from mmla_audio_amd import _lib, weights  # noqa: E402
from oracle import synth  # noqa: E402


lib = _lib.load_library(sys.argv[1])
ctx = _lib.Context(0)
W = weights.synthetic(weights.OD, seed=0)
ctx.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
pcm = synth.batch(1, 4096, 40000)
LAYERS = [(3, 3, 64, 32, 64), (4, 1, 64, 64, 64), (3, 3, 32, 64, 64), (4, 1, 32, 64, 64),
          (3, 3, 32, 64, 128), (4, 1, 32, 128, 128), (3, 3, 16, 128, 128), (4, 1, 16, 128, 128)]
names = ['prologue', 'stage', 'barrier', 'taps', 'epilogue', 'total']
for sel in LAYERS:
    lib.mmla_debug_conv_select(*sel)
    ctx.od_pipeline(pcm)
    buf = (ctypes.c_ulonglong * (8192 * 4 * 8))()
    lib.mmla_debug_conv_times(buf)
    t = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 4, 8).astype(np.int64)
    ok = t[:, :, 5] > 0
    if not ok.any():
        print(sel, 'no samples')
        continue
    med = [int(np.median(t[:, :, i][ok])) for i in range(6)]
    start = t[:, :, 7][ok]
    life = t[:, :, 5][ok]
    span = (start + life).max() - start.min()
    print('kh,kw,h,cin,cout', sel, 'chunks', int(np.median(t[:, :, 6][ok])),
          ' '.join(f'{n}={m}' for n, m in zip(names, med)),
          f'concurrent waves ~{life.sum() / span / 4:.1f} per CU-slot-4')
