"""CPU: the N>1 driver logic (sharding + logits all-gather) with world_size 2 over gloo."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mmla_audio_amd.distributed import gather_logits, shard_range


def test_shard_range_covers_batch():
    for n in (0, 1, 7, 65536, 524288, 1001):
        for w in (1, 2, 4, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, ret):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    lo, hi = shard_range(n_total, rank, world)
    # each rank's "probabilities" encode the global clip index so order is checkable
    local = torch.stack([torch.arange(lo, hi, dtype=torch.float32),
                         -torch.arange(lo, hi, dtype=torch.float32)], dim=1)
    full = gather_logits(local, n_total)
    ret[rank] = full.clone()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('n_total', [64, 67])
def test_gather_logits_two_ranks_gloo(n_total):
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, port, n_total, ret), nprocs=world, join=True)
    want = torch.stack([torch.arange(n_total, dtype=torch.float32),
                        -torch.arange(n_total, dtype=torch.float32)], dim=1)
    for r in range(world):
        assert torch.equal(ret[r], want)
