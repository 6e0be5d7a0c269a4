"""Dev A/B check: OD / SI pipeline probabilities of one library build on a fixed synthetic batch.

python tools/lib_probs.py <libmmla.so> <out.npy> [od|si] [clips]
Two runs (two processes, two builds) whose .npy files are equal byte for byte produced bit-identical
network outputs.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    lib, out = sys.argv[1], sys.argv[2]
    which = sys.argv[3] if len(sys.argv) > 3 else 'od'
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
    import torch
    from mmla_audio_amd import _lib, weights
    from mmla_audio_amd.synthetic import make_clips
    _lib.load_library(lib)
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    clip_len = 40000 if which == 'od' else 24000
    if which == 'od':
        spec, K = weights.OD, 2
        ctx.load_weights(spec, weights.pack(spec, weights.synthetic(spec, seed=0)), K)
    else:
        spec, K = weights.SI, 630
        ctx.load_weights(spec, weights.pack(spec, weights.synthetic(spec, seed=0, n_classes=K), K), K,
                         _lib.HEAD_SOFTMAX)
    pcm = make_clips(n, clip_len, start_index=0)
    probs = torch.empty((n, K), dtype=torch.float32, device='cuda')
    am = torch.empty(n, dtype=torch.int32, device='cuda')
    run = ctx.od_pipeline_dev if which == 'od' else ctx.si_pipeline_dev
    run(pcm.data_ptr(), n, clip_len, clip_len, probs.data_ptr(), am.data_ptr())
    torch.cuda.synchronize()
    np.save(out, probs.cpu().numpy())
    print(which, n, 'clips ->', out)


if __name__ == '__main__':
    main()
