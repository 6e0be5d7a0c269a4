"""Per-phase cycle totals of the OD front-end (dev tool).

Needs the instrumented library: `make -C mmla_audio_amd/csrc exp` builds
mmla_audio_amd/libmmla_exp.so with -DFE_EXP=1.  MMLA_FE_IMPL=1 selects the v1 kernel.
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, '.')
from mmla_audio_amd import _lib  # noqa: E402
from oracle import synth  # noqa: E402

path = os.path.join(os.path.dirname(_lib.LIB_PATH), 'libmmla_exp.so')
lib = _lib.load_library(path)
ctx = _lib.Context(0)
pcm = synth.batch(0, 4096, 40000)
ctx.od_features(pcm, db=False, zcr=False, img=False)
ctx.od_features(pcm, db=False, zcr=False, img=False)
buf = (ctypes.c_ulonglong * (4096 * 8))()
lib.mmla_debug_fe_times(buf)
t = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.float64)
if os.environ.get('MMLA_FE_IMPL') == '1':
    names = ['window+wait', 'zcr', 'pass1', 'pass2a', 'pass2b', 'mel', 'epilogue']
else:
    names = ['window+wait', 'zcr', 'passA', 'passB', 'split', 'mel+store', 'epilogue']
tot = t[:, :7].sum(1)
print('median clip cycles', np.median(tot))
for i in range(7):
    print(f'  {names[i]:12s} {np.median(t[:, i]):10.0f}  {100 * np.median(t[:, i] / tot):5.1f}%')
