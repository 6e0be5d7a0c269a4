"""BASELINE config 5 on one card: two ranks (processes) share cuda:0, each runs its contiguous shard
through the fused pipeline (mmla_audio_amd.distributed.sharded_predict), the shards' probabilities
are all-gathered (gloo here; RCCL over xGMI in bench.py on a node), and the gathered [n, K] must
equal the single-process run bit for bit (clips are independent, no data-path exchange).
"""
import os
import socket

import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu

N_OD, N_SI = 67, 45   # ragged shards (34 + 33, 23 + 22)


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _weights():
    from mmla_audio_amd import weights
    return (weights.synthetic(weights.OD, seed=91),
            weights.synthetic(weights.SI, seed=92, n_classes=8))


def _load(ctx):
    from mmla_audio_amd import weights
    w_od, w_si = _weights()
    ctx.load_weights(weights.OD, weights.pack(weights.OD, w_od), 2)
    ctx.load_weights(weights.SI, weights.pack(weights.SI, w_si, 8), 8, 1)


def _inputs():
    return synth.batch(4000, N_OD, 40000), synth.batch(4100, N_SI, 24000)


def _conversation():
    """~33 s conversation: 13 windows of 256 frames (7 + 6 per rank), a partial last window"""
    return np.concatenate([synth.clip(4200 + k, 40960) for k in range(13)])[:13 * 256 * 160 - 5000]


def _rank(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from mmla_audio_amd import _lib
    from mmla_audio_amd.distributed import sharded_predict
    ctx = _lib.Context(0)
    _load(ctx)
    od, si = _inputs()
    p_od = sharded_predict(od, 0, ctx, rank, world, on_device=False)
    p_si = sharded_predict(si, 1, ctx, rank, world, on_device=False)
    np.save(os.path.join(out_dir, f'od_{rank}.npy'), p_od.numpy())
    np.save(os.path.join(out_dir, f'si_{rank}.npy'), p_si.numpy())
    from mmla_audio_amd.distributed import conversation_features_shard, sharded_conversation_predict
    conv = _conversation()
    np.save(os.path.join(out_dir, f'convfeat_{rank}.npy'),
            conversation_features_shard(conv, rank, world, ctx.si_features_seq))
    np.save(os.path.join(out_dir, f'conv_{rank}.npy'),
            sharded_conversation_predict(conv, ctx, rank, world, on_device=False).numpy())
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


def test_two_ranks_on_one_gpu_match_single_process(tmp_path):
    import torch.multiprocessing as mp
    from mmla_audio_amd import _lib
    mp.spawn(_rank, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    ctx = _lib.Context(0)
    _load(ctx)
    od, si = _inputs()
    ref_od, _, _ = ctx.od_pipeline(od)
    ref_si, _, _ = ctx.si_pipeline(si)
    for r in range(2):
        assert np.array_equal(np.load(tmp_path / f'od_{r}.npy'), ref_od)
        assert np.array_equal(np.load(tmp_path / f'si_{r}.npy'), ref_si)
    # SI whole-conversation mode sharded by window range (distributed.sharded_conversation_predict):
    # each rank's windows from its own slice + halo equal the single-process windows bit for bit
    conv = _conversation()
    whole = ctx.si_features_seq(conv)
    assert np.array_equal(np.concatenate([np.load(tmp_path / f'convfeat_{r}.npy') for r in range(2)]),
                          whole)
    ref_conv = ctx.si_forward(whole)
    for r in range(2):
        assert np.array_equal(np.load(tmp_path / f'conv_{r}.npy'), ref_conv)
