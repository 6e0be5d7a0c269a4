"""Per-phase cycle totals of the OD front-end (dev tool; library built with -DFE_EXP=1)."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, '.')
from mmla_audio_amd import _lib  # noqa: E402
from oracle import synth  # noqa: E402

ctx = _lib.Context(0)
pcm = synth.batch(0, 4096, 40000)
ctx.od_features(pcm, db=False, zcr=False, img=False)
ctx.od_features(pcm, db=False, zcr=False, img=False)
buf = (ctypes.c_ulonglong * (4096 * 8))()
ctypes.CDLL(_lib.LIB_PATH).mmla_debug_fe_times(buf)
t = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.float64)
names = ['window+wait', 'zcr', 'pass1', 'pass2a', 'pass2b', 'mel', 'epilogue', '-']
tot = t[:, :7].sum(1)
print('median clip cycles', np.median(tot))
for i in range(7):
    print(f'  {names[i]:12s} {np.median(t[:, i]):10.0f}  {100 * np.median(t[:, i] / tot):5.1f}%')
