"""Per-phase cycles of the MFMA OD front-end (od_fe.hip v3) -- dev tool.

Needs the instrumented library: `make -C mmla_audio_amd/csrc exp` builds libmmla_exp.so with
-DFE_EXP=1 (s_memtime per interval of the step pipeline, per wave, summed over a clip's 5 steps).
Usage: python tools/fe3_timeline.py [waves_per_workgroup=8]
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from mmla_audio_amd import _lib  # noqa: E402
from oracle import synth  # noqa: E402

nwv = int(sys.argv[1]) if len(sys.argv) > 1 else 8
lib = _lib.load_library(os.environ.get('FE3_LIB', os.path.join(os.path.dirname(_lib.LIB_PATH), 'libmmla_exp.so')))
ctx = _lib.Context(0)
pcm = synth.batch(0, 4096, 40000)
for _ in range(3):
    ctx.od_features(pcm, db=False, zcr=True, img=False)
buf = (ctypes.c_ulonglong * (4096 * 8))()
lib.mmla_debug_fe_times(buf)
nclip = 4096 // nwv
t = np.frombuffer(buf, dtype=np.uint64).reshape(nclip, nwv, 8).astype(np.float64)
names = ['A: s1+mel', 'A barrier', 'B: s2+stage', 'B barrier', 'epilogue', '-', '-', '-']
tot = t.sum(2)
print(f'{nwv} waves/workgroup: median cycles per clip (wave 0) {np.median(tot[:, 0]):.0f}, '
      f'max over waves {np.median(tot.max(1)):.0f}')
for i, n in enumerate(names):
    med = np.median(t[:, :, i], axis=0)
    print(f'  {n:11s} ' + ' '.join(f'{v:7.0f}' for v in med))
