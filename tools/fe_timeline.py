"""Dev tool: phase timeline of the OD front-end (od_fe3_kernel<false, true, false>, the config-2 norm
output) from an FE_TRACE build (make variant ... VDEF="-DFE_TRACE=1 ..."; with -DFE_INPLACE=1 on the
in-place dB dev copy for VERDICT r5 #2).
python tools/fe_timeline.py <libmmla_trace.so> [label]
The trace holds every tile step of the third clip of the first 256 workgroups (16 waves each); the
software pipeline's two intervals per step are (od_fe.hip, the loop in od_fe3_kernel):
  A: crossings + stage 1 of tile t  |  at t = 1: the previous clip's epilogue (max / min -> norm)
  B: mel of tile t - 1  |  stage 2 of tile t  |  ZCR sum + staging of tile t + 1 + its prefetch"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mmla_audio_amd import _lib  # noqa: E402
from oracle import synth  # noqa: E402

lib = _lib.load_library(sys.argv[1])
label = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(sys.argv[1])
ctx = _lib.Context(0)
pcm = synth.batch(1234, 4096, 24000)
for _ in range(2):
    ctx.od_features(pcm, db=False, norm=True, zcr=True, img=False)
buf = np.zeros(256 * 16 * 5 * 8, np.uint64)
fn = lib.mmla_debug_fe_trace
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
t = buf.reshape(256, 16, 5, 8).astype(np.int64)
ok = t[..., 7] > 0
d = np.diff(t, axis=-1)                          # [wg, wave, tile, 7]
names = ['A: crossings+stage1', 'A: epilogue', 'barrier A', 'B: mel(t-1)', 'B: stage2', 'B: zcr+staging',
         'barrier B']
out = {'label': label, 'samples': int(ok.sum()), 'unit': 'shader clock cycles (s_memtime)',
       'step_median': float(np.median((t[..., 7] - t[..., 0])[ok]))}
for tile_set, tag in (((0, 2, 3, 4), 'tiles without the epilogue'), ((1,), 'tile 1 (with the epilogue)')):
    m = ok[:, :, list(tile_set)]
    dd = d[:, :, list(tile_set)][m]
    out[tag] = {n: {'median': float(np.median(dd[:, i])), 'p90': float(np.percentile(dd[:, i], 90))}
                for i, n in enumerate(names)}
print(json.dumps(out, indent=1))
