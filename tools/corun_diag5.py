"""dev: does any kernel of context b write into context a's memory?  a's front-end scratch slot and a
torch tensor are filled with 0x5A; b then runs OD-NET stage by stage (debug trace), the whole net,
the pipeline and the front-end, each alone and synchronised; after each the canaries are checked."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mmla_audio_amd import _lib, weights  # noqa: E402
from oracle import synth  # noqa: E402

W = weights.synthetic(weights.OD, seed=41)
N = 1024
hip = ctypes.CDLL('libamdhip64.so')


def ctx():
    c = _lib.Context(0)
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    c.set_microbatch(128, 128)
    return c


def slot(c, k):
    p, b = ctypes.c_void_p(), ctypes.c_size_t()
    assert c.lib.mmla_debug_ws_slot(c.h, k, ctypes.byref(p), ctypes.byref(b)) == 0
    return p.value, b.value


def main():
    od = torch.from_numpy(synth.batch(990, N, 40000)).cuda()
    img0 = torch.zeros((N, 128, 151, 3), dtype=torch.uint8, device='cuda')
    a = ctx()
    a.od_features_dev(od.data_ptr(), N, 40000, 40000, img=img0.data_ptr())
    torch.cuda.synchronize()
    sp, sb = slot(a, 17)   # S_FESCR
    canary = torch.full((N * 128 * 151 * 3,), 0x5A, dtype=torch.uint8, device='cuda')
    print(f'a scratch slot at {sp:#x}, {sb} B; canary tensor at {canary.data_ptr():#x}', flush=True)
    host = np.empty(sb, np.uint8)

    def arm():
        assert hip.hipMemset(ctypes.c_void_p(sp), 0x5A, ctypes.c_size_t(sb)) == 0
        canary.fill_(0x5A)
        torch.cuda.synchronize()

    def check(tag):
        torch.cuda.synchronize()
        assert hip.hipMemcpy(host.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(sp),
                             ctypes.c_size_t(sb), 2) == 0
        bad = np.nonzero(host != 0x5A)[0]
        cb = torch.nonzero(canary != 0x5A).flatten().cpu().numpy()
        msg = f'{tag:28s} scratch bytes hit {len(bad):9d}'
        if len(bad):
            msg += f' [{bad[0]:#x} .. {bad[-1]:#x}]'
        msg += f' | canary bytes hit {len(cb):9d}'
        if len(cb):
            msg += f' [{cb[0]:#x} .. {cb[-1]:#x}]'
        print(msg, flush=True)

    b = ctx()
    x = img0[:128].cpu().numpy().astype(np.float32)
    arm()
    check('nothing run')
    for stage in range(12):
        arm()
        b.debug_od_trace(x, stage)
        check(f'b trace stage {stage}')
    for name, fn in (('b net', lambda: b.od_forward_dev(img0.data_ptr(), N, canary.data_ptr() * 0 or _probs.data_ptr(), u8=True)),
                     ('b pipeline', lambda: b.od_pipeline_dev(od.data_ptr(), N, 40000, 40000, _probs.data_ptr())),
                     ('b front-end', lambda: b.od_features_dev(od.data_ptr(), N, 40000, 40000, img=_img.data_ptr())),
                     ('a net (own scratch)', lambda: a.od_forward_dev(img0.data_ptr(), N, _probs.data_ptr(), u8=True))):
        for it in range(2):
            arm()
            fn()
            check(f'{name} #{it}')


_probs = torch.zeros((N, 2), device='cuda')
_img = torch.zeros((N, 128, 151, 3), dtype=torch.uint8, device='cuda')

if __name__ == '__main__':
    main()
