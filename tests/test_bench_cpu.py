"""CPU: bench.py's host logic -- the --gpus N launcher (ranks started under torch.distributed.run
before any GPU call), the parity-sample indices, and the CPU-baseline helpers."""
import os
import sys

import pytest

import bench


def test_gpus_n_launches_torchrun(monkeypatch):
    calls = []
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '4', '--steps', '2'])
    monkeypatch.setattr(bench.subprocess, 'call', lambda cmd, env=None: calls.append((cmd, env)) or 7)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    cmd, env = calls[0]
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--nproc-per-node=4' in cmd and '127.0.0.1' in cmd
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert os.path.basename(cmd[cmd.index('--master-port') + 2]) == 'bench.py'
    assert cmd[-4:] == ['--gpus', '4', '--steps', '2']
    assert env['MASTER_ADDR'] == '127.0.0.1'


def test_sample_covers_microbatch_edges():
    idx = bench.sample_indices(65536, 16384, 24)
    for c0 in range(0, 65536, 16384):
        assert c0 in idx and c0 + 16383 in idx
    assert len(idx) >= 24 and idx == sorted(set(idx))
    assert bench.sample_indices(5, 16384, 24) == [0, 1, 2, 3, 4]


def test_cpu_baseline_host_info():
    from oracle import cpu_baseline
    h = cpu_baseline.host_info()
    assert h['os_cpu_count'] >= 1 and h['affinity_cpus'] >= 1 and h['affinity']
    assert cpu_baseline._ranges([0, 1, 2, 5, 7, 8]) == '0-2,5,7-8'
    assert 1 <= cpu_baseline.usable_cores() <= h['affinity_cpus']
