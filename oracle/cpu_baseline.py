"""CPU baselines for bench.py (SURVEY.md 8(d) "CPU baseline timed beside it") -- TEST
INFRASTRUCTURE ONLY: the oracle restatements timed on the host cores, never the product path.

Two modes, each in its own child process so that core pinning and thread pools do not leak into the
GPU process (bench.py runs them before it touches the GPU):
  faithful   the reference's shape: one clip at a time, front-end -> (OD: image quantisation ->)
             network, on ONE pinned core with every thread pool at 1 (record_on_pc.py:114-171,
             SI record_on_pc.py:97-140).  numpy librosa-0.8 / psf-0.6 restatements + numpy float32
             nets (oracle/od_fe.py, si_fe.py, nets.py).
  best       best effort on the host cores this GPU's job may use: the front-end in a process pool
             (one clip per task), then the torch-CPU float32 nets (oracle/nets_torch.py) batched
             with torch threads = cores.  The pool is sized to the job's CPU share (OMP_NUM_THREADS,
             16 per GPU on the MI355X pool -- the operators' rule for pool sizes on a shared box), not
             to every core of the host; host_info() records both counts, so the line says exactly
             what was timed.
Workloads: od_pipeline, si_pipeline, od_features (front-end only), noise_gate.
Inputs are oracle/synth clips (the SURVEY 8(d) five-class recipe bench.py generates on the GPU).
"""
import os
import platform
import queue
import time

import numpy as np


def host_info():
    model = platform.processor() or ''
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    aff = sorted(os.sched_getaffinity(0))
    return {'cpu_model': model, 'os_cpu_count': os.cpu_count(), 'affinity_cpus': len(aff),
            'affinity': _ranges(aff), 'physical_cores': physical_cores(aff),
            'omp_num_threads': os.environ.get('OMP_NUM_THREADS')}


def physical_cores(cpus):
    """distinct (package, core) pairs among the logical CPUs `cpus` (SMT siblings count once)"""
    seen = set()
    for c in cpus:
        base = f'/sys/devices/system/cpu/cpu{c}/topology/'
        try:
            with open(base + 'physical_package_id') as f:
                pkg = f.read().strip()
            with open(base + 'core_id') as f:
                core = f.read().strip()
        except OSError:
            return len(cpus)
        seen.add((pkg, core))
    return len(seen)


def _ranges(cpus):
    out, start, prev = [], None, None
    for c in cpus:
        if start is None:
            start = prev = c
        elif c == prev + 1:
            prev = c
        else:
            out.append(f'{start}-{prev}' if start != prev else f'{start}')
            start = prev = c
    if start is not None:
        out.append(f'{start}-{prev}' if start != prev else f'{start}')
    return ','.join(out)


def usable_cores():
    """physical cores of the affinity set, capped by the job's CPU share (OMP_NUM_THREADS)"""
    n = physical_cores(sorted(os.sched_getaffinity(0)))
    omp = os.environ.get('OMP_NUM_THREADS')
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, n)


def _weights(workload):
    from mmla_audio_amd import weights
    if workload == 'od_pipeline':
        return weights.synthetic(weights.OD, seed=0)
    if workload == 'si_pipeline':
        return weights.synthetic(weights.SI, seed=0, n_classes=630)
    return None


def _clip_len(workload):
    return 24000 if workload == 'si_pipeline' else 40000


def _noise():
    return (0.01 * np.random.default_rng(4242).standard_normal(160000)).astype(np.float32)


def _clips(workload, start, n):
    """the sample, synthesised before any timing starts"""
    from oracle import synth
    return [synth.clip(start + i, _clip_len(workload)) for i in range(n)]


def _fe_one(args):
    """front-end of one clip (pool task): OD -> image (or norm for od_features), SI -> [256,39]"""
    workload, pcm = args
    if workload == 'si_pipeline':
        from oracle import si_fe
        return si_fe.input_feature_gen(pcm)[0].astype(np.float32)
    if workload == 'noise_gate':
        from oracle import noisereduce as onr
        return onr.reduce_noise((pcm / 32768.0).astype(np.float32), 16000, _noise())
    from oracle import od_fe
    f = od_fe.od_features(pcm)
    return f['png_rgb'].astype(np.float32) if workload == 'od_pipeline' else f['norm']


def _limit_threads(n):
    from threadpoolctl import threadpool_limits
    threadpool_limits(n)
    try:
        import torch
        torch.set_num_threads(n)
    except ImportError:
        pass


def _pool_init():
    _limit_threads(1)


def faithful(workload, budget_s, start=0, q=None):
    """serial batch-1 loop on one pinned core"""
    cpu = sorted(os.sched_getaffinity(0))[0]
    os.sched_setaffinity(0, {cpu})
    _limit_threads(1)
    from oracle import nets
    W = _weights(workload)
    sample = _clips(workload, start, 16)
    _fe_one((workload, sample[0]))        # imports / table builds outside the timed loop
    n, t0 = 0, time.perf_counter()
    while True:
        x = _fe_one((workload, sample[n % len(sample)]))
        if workload == 'od_pipeline':
            nets.od_forward(x[None], W, dtype=np.float32)
        elif workload == 'si_pipeline':
            nets.si_forward(x[None], W, dtype=np.float32)
        n += 1
        dt = time.perf_counter() - t0
        if dt > budget_s:
            break
    res = {'value': n / dt, 'clips': n, 'seconds': dt, 'cores': 1, 'pinned_cpu': cpu}
    if q is not None:
        q.put(res)
    return res


def best(workload, budget_s, start=0, q=None):
    """process-pool front-end + batched torch-CPU nets on all usable cores"""
    import multiprocessing as mp
    cores = usable_cores()
    _limit_threads(cores)
    nt = None
    W = _weights(workload)
    if W is not None:
        from oracle.nets_torch import Nets
        import torch
        nt = Nets(W, dtype=torch.float32)
    chunk = max(cores * 2, 16)
    sample = _clips(workload, start, chunk)
    with mp.get_context('spawn').Pool(cores, initializer=_pool_init) as pool:
        # pool start-up and the workers' first imports are outside the timed loop
        pool.map(_fe_one, [(workload, sample[j % chunk]) for j in range(cores)], chunksize=1)
        if nt is not None:
            x0 = np.stack([_fe_one((workload, sample[0]))] * 2)
            nt.od_forward(x0) if workload == 'od_pipeline' else nt.si_forward(x0)
        n, t0 = 0, time.perf_counter()
        while True:
            xs = pool.map(_fe_one, [(workload, p) for p in sample], chunksize=1)
            if workload == 'od_pipeline':
                nt.od_forward(np.stack(xs))
            elif workload == 'si_pipeline':
                nt.si_forward(np.stack(xs))
            n += chunk
            dt = time.perf_counter() - t0
            if dt > budget_s:
                break
    res = {'value': n / dt, 'clips': n, 'seconds': dt, 'cores': cores, 'batch': chunk}
    if q is not None:
        q.put(res)
    return res


def run_modes(workload, budget_s):
    """both modes, each in a spawned child process; -> cpu_baseline dict for the bench line"""
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    out = {}
    for name, fn, b in (('faithful_1core', faithful, 0.4 * budget_s), ('best_job_cores', best, 0.6 * budget_s)):
        q = ctx.Queue()
        p = ctx.Process(target=fn, args=(workload, b, 0, q))
        p.start()
        try:
            t0 = time.time()
            while name not in out:
                try:
                    out[name] = q.get(timeout=2)
                except queue.Empty:
                    if not p.is_alive() or time.time() - t0 > b + 300:
                        raise RuntimeError(f'CPU baseline {name} ({workload}) died or hung '
                                           f'(exit code {p.exitcode})')
        finally:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    what = {
        'od_pipeline': 'OD front-end (numpy librosa-0.8 restatement) -> quantised image -> OD-NET',
        'si_pipeline': 'SI front-end (numpy python_speech_features-0.6 restatement) -> SI-NET (K=630)',
        'od_features': 'OD front-end only (numpy librosa-0.8 restatement: log-mel norm + ZCR)',
        'noise_gate': 'noisereduce-2.0 stationary gate (numpy librosa-0.8 stft/istft + scipy '
                      'fftconvolve restatement)',
    }[workload]
    bb, ff = out['best_job_cores'], out['faithful_1core']
    host = host_info()
    return {
        'value': bb['value'], 'unit': 'clips/s', 'cores': bb['cores'], 'kind': 'port',
        'sample': f"{bb['clips']} synthetic {_clip_len(workload) / 16000:g} s clips (oracle/synth, the "
                  f"SURVEY 8(d) five-class recipe): {what}; value = mode best_job_cores "
                  f"(process-pool front-end + batched torch-CPU float32 nets on {bb['cores']} cores = "
                  f"this job's CPU share; the host has {host['physical_cores']} physical cores in "
                  f"the affinity set, {host['affinity_cpus']} logical); faithful_1core = the "
                  f"reference's batch-1 loop on one pinned core ({ff['clips']} clips, {ff['value']:.2f} "
                  f"clips/s, numpy float32 nets)",
        'modes': out, 'host': host,
    }
