"""Phase timeline of the fused res_block kernel (dev tool): needs a library built with
-DRB_EXP=4 (s_memtime marks of the first 8192 workgroups of the pool-block launch)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, '.')
from mmla_audio_amd import _lib, weights  # noqa: E402

LIB = os.environ.get('MMLA_LIB', _lib.LIB_PATH)   # a -DRB_EXP=4 build
_lib.load_library(LIB)

ctx = _lib.Context(0)
W = weights.synthetic(weights.OD, seed=0)
ctx.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
n = 4096
rng = np.random.default_rng(0)
img = rng.integers(0, 256, size=(n, 128, 151, 3), dtype=np.uint8)
ctx.od_forward(img)
ctx.od_forward(img)
buf = (ctypes.c_ulonglong * (8192 * 4 * 8))()
lib = ctypes.CDLL(LIB)
rc = lib.mmla_debug_resblk_times(buf)
t = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 4, 8).astype(np.int64)
t0 = t[:, :, 0].min()
t = t - t0
names = ['load+w2', 'stage', 'gemm1', 'bar', 'phaseB', 'gemm2', 'epilogue']
d = np.diff(t, axis=2)            # [wg, wave, 7]
print('rc', rc, 'median phase cycles (over wg x wave):')
for i, nm in enumerate(names):
    print(f'  {nm:9s} med {np.median(d[:, :, i]):8.0f}  p10 {np.percentile(d[:, :, i], 10):8.0f}  p90 {np.percentile(d[:, :, i], 90):8.0f}')
life = t[:, :, 7].max(1) - t[:, :, 0].min(1)
print('wg lifetime med', np.median(life), 'p90', np.percentile(life, 90))
start = t[:, :, 0].min(1)
end = t[:, :, 7].max(1)
span = end.max() - start.min()
print('span of 8192 WGs (cycles)', span, ' -> WG-cycles / span =', life.sum() / span, 'concurrent WGs on average')
# launch cadence
ss = np.sort(start)
print('start quantiles', [int(x) for x in np.percentile(ss, [0, 1, 5, 25, 50, 75, 100])])
