"""Dev tool: phase timeline of the rbs strip kernels from an RBS_TRACE build (make variant VDEF=-DRBS_TRACE=1).
python tools/rbs_timeline.py <libmmla_trace.so> [block: 1 | 2]
Runs the debug trace on 2048 clips with MMLA_RB_TILE unset; the trace holds the LAST launch of
the strip kernels that ran (block 1 only, when run with --upto 1 via debug trace stage 1)."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mmla_audio_amd import _lib, weights  # noqa: E402
from oracle import synth  # noqa: E402

lib = _lib.load_library(sys.argv[1])
stage = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ctx = _lib.Context(0)
W = weights.synthetic(weights.OD, seed=0)
ctx.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
x = np.random.default_rng(0).integers(0, 256, size=(2048, 128, 151, 3)).astype(np.float32)
for _ in range(2):
    ctx.debug_od_trace(x, stage)
buf = np.zeros(2048 * 4 * 4 * 8, np.uint64)
fn = lib.mmla_debug_rbs_trace
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
t = buf.reshape(2048, 4, 4, 8).astype(np.int64)
ok = t[..., 7] > 0
d = np.diff(t, axis=-1)[ok]          # [samples, 7]
names = ['staging', 'barrier1', 'gemm1', 't1_write+loads', 'barrier2', 'gemm2', 'epilogue']
tot = (t[..., 7] - t[..., 0])[ok]
print(f'block stage {stage}: {ok.sum()} (wg, wave, chunk) samples, chunk median {np.median(tot):.0f} cycles')
for i, n in enumerate(names):
    print(f'  {n:16s} median {np.median(d[:, i]):7.0f}  p90 {np.percentile(d[:, i], 90):7.0f}')
# chunk-to-chunk gap (loop overhead)
