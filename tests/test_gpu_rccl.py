"""The RCCL path of SURVEY 8(e) executed on the MI355X at world size 1 (VERDICT r5 missing #2):
``init_process_group('nccl', device_id=...)`` in-process (no re-exec, rendezvous on 127.0.0.1), then
``distributed.gather_logits`` through ``all_gather_into_tensor`` (equal shards) and the size
exchange + ``all_gather`` (ragged) on device tensors the library wrote -- once on the context's own
blocking stream, once on torch's current stream handed over with ``set_stream`` (bench.py's
arrangement).  The gathered probabilities must equal a host-pointer call on the same clips bit for
bit.  The multi-rank arithmetic of the same function is covered on gloo by
test_distributed_cpu.py / test_gpu_sharded.py."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture()
def nccl_group():
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip('a process group is already initialised in this process')
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(_free_port())
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    assert dist.get_backend() == 'nccl'
    try:
        yield dist
    finally:
        dist.destroy_process_group()


def test_rccl_gather_of_library_outputs(nccl_group):
    from mmla_audio_amd import _lib, weights
    from mmla_audio_amd.distributed import gather_logits
    from mmla_audio_amd.synthetic import make_clips
    n = 37
    ctx = _lib.Context(0)
    ctx.load_weights(weights.OD, weights.pack(weights.OD, weights.synthetic(weights.OD, seed=3)), 2)
    pcm = make_clips(n, 40000, start_index=900)
    torch.cuda.synchronize()
    ref, ref_am, _ = ctx.od_pipeline(np.ascontiguousarray(pcm.cpu().numpy()))

    for handover in (False, True):
        if handover:
            ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        probs = torch.full((n, 2), float('nan'), dtype=torch.float32, device='cuda')
        am = torch.full((n,), -7, dtype=torch.int32, device='cuda')
        # written on the library's stream (its own blocking stream, or torch's after the handover);
        # no host synchronisation before the collectives
        ctx.od_pipeline_dev(pcm.data_ptr(), n, 40000, 40000, probs.data_ptr(), am.data_ptr())
        out = torch.empty_like(probs)
        got = gather_logits(probs, n_total=n, out=out, force_collective=True)
        assert got is out
        ragged = gather_logits(probs[:5], force_collective=True)       # size exchange path
        am_all = gather_logits(am[:, None], n_total=n, force_collective=True)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ref), f'handover={handover}'
        assert np.array_equal(ragged.cpu().numpy(), ref[:5])
        assert np.array_equal(am_all[:, 0].cpu().numpy(), ref_am)
    ctx.set_stream(None)


def test_rccl_world1_barrier_and_max(nccl_group):
    """bench.py's barrier + max-over-ranks collectives on the nccl group"""
    dist = nccl_group
    dist.barrier()
    t = torch.tensor([1.5], dtype=torch.float64, device='cuda')
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert float(t.item()) == 1.5
