#!/usr/bin/env python3
"""Benchmark: audio clips/s (MFCC -> logits) on 1..8 MI355X, one process per GPU.

  python bench.py [--gpus N --steps K --warmup W --workload od_pipeline|si_pipeline|od_features]
  torchrun --nproc-per-node N ... bench.py --gpus N   (RCCL all-gather of the logits per step)

A step = one pass of the hot path over one batch of synthetic clips already resident in HBM:
  od_pipeline (default, BASELINE config 3): 65 536 x 2.5 s clips / GPU, fused log-mel+ZCR front-end
      -> quantised image -> OD-NET (Conv2D ResNet + BiLSTM + Dense) -> softmax/argmax;
      at N GPUs the per-shard probabilities are all-gathered over RCCL (config 5 at N = 8).
  si_pipeline (config 4): 65 536 x 1.5 s clips / GPU, MFCC+delta+delta-delta -> SI-NET, K = 630.
  od_features (config 2): the front-end kernel alone, 4 096 x 2.5 s clips / GPU.
Prints ONE JSON line (rank 0) with roofline + cpu_baseline objects.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = 'audio clips/sec (MFCC→logits) at 1/2/4/8 MI355X; MFCC max-abs-err vs librosa'
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
F32_MFMA_PEAK_TFS = 157.3    # v_mfma_f32_32x32x2_f32, dense
F16_MFMA_PEAK_TFS = 2516.6   # f16 MFMA dense (~2.5 PF spec, no sparsity)
# 3xFP16 spends three f16 MFMA products per f32 MAC: its f32-equivalent ceiling is F16 / 3
F16X3_PEAK_TFS = F16_MFMA_PEAK_TFS / 3
OD_FE_BYTES = 48000 + 128 * 151 * 4 + 151 * 4          # 125 916 B/clip


def pmc_traffic(workload, stage, clips):
    """HBM bytes per launch of `stage` from the committed PMC capture of this workload
    (tools/gpu/pmc_traffic.sh -> profiles/pmc_traffic_<workload>.json), scaled to this run's clips
    per launch; None when no capture exists."""
    path = os.path.join(REPO, 'profiles', f'pmc_traffic_{workload}.json')
    try:
        d = json.load(open(path))
        st = d['stages'][stage]
        per_clip = st['traffic_bytes_per_launch'] / d['clips_per_launch'][stage]
        return per_clip * min(clips, d['clips_per_launch'][stage]), os.path.relpath(path, REPO)
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--workload', default='od_pipeline',
                    choices=['od_pipeline', 'si_pipeline', 'od_features', 'noise_gate'])
    ap.add_argument('--clips', type=int, default=None, help='clips per GPU')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--microbatch', type=int, default=0,
                    help='clips per internal micro-batch (0 = the library default)')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    return ap.parse_args()


def dist_setup():
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        torch.cuda.set_device(local)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device='cuda')
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline_od(pcm_sample, gpu_norm, gpu_probs, W, budget_s):
    """Oracle (numpy) FE + OD-NET on a bounded sample of the same clips, on the host cores."""
    from oracle import nets, od_fe
    threads = int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1))
    n_done = 0
    err_norm = 0.0
    err_prob = 0.0
    t0 = time.perf_counter()
    for i in range(len(pcm_sample)):
        f = od_fe.od_features(pcm_sample[i])
        p = nets.od_forward(f['png_rgb'][None].astype(np.float32), W, dtype=np.float32)
        ok = ~np.isnan(f['norm'])
        if ok.any():
            err_norm = max(err_norm, float(np.abs(gpu_norm[i][ok] - f['norm'][ok]).max()))
        err_prob = max(err_prob, float(np.abs(gpu_probs[i] - p[0]).max()))
        n_done += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {'value': n_done / dt, 'unit': 'clips/s', 'cores': threads, 'kind': 'port',
            'sample': f'{n_done} x 2.5 s synthetic clips, batch 1 (record_on_pc.py loop shape): '
                      f'numpy librosa-0.8 restatement + numpy float32 OD-NET (BLAS threads={threads})'}, \
        err_norm, err_prob


def cpu_baseline_nr(y_sample, noise, gpu_out, budget_s):
    """Oracle (numpy/scipy) noisereduce-2.0 stationary gate on a bounded sample of the clips."""
    from oracle import noisereduce as onr
    threads = int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1))
    n_done, err = 0, 0.0
    t0 = time.perf_counter()
    for i in range(len(y_sample)):
        w = onr.reduce_noise(y_sample[i], 16000, noise)
        err = max(err, float(np.abs(gpu_out[i] - w).max()))
        n_done += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {'value': n_done / dt, 'unit': 'clips/s', 'cores': threads, 'kind': 'port',
            'sample': f'{n_done} x 2.5 s synthetic clips, one call each (record_on_pc.py shape): numpy '
                      f'librosa-0.8 stft/istft + scipy fftconvolve restatement of noisereduce 2.0 '
                      f'(BLAS threads={threads})'}, err


def cpu_baseline_si(pcm_sample, gpu_feat, gpu_probs, W, budget_s):
    from oracle import nets, si_fe
    threads = int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1))
    n_done = 0
    err_feat = 0.0
    err_prob = 0.0
    t0 = time.perf_counter()
    for i in range(len(pcm_sample)):
        x = si_fe.input_feature_gen(pcm_sample[i])
        p = nets.si_forward(x.astype(np.float32), W, dtype=np.float32)
        err_feat = max(err_feat, float(np.abs(gpu_feat[i] - x[0]).max()))
        err_prob = max(err_prob, float(np.abs(gpu_probs[i] - p[0]).max()))
        n_done += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {'value': n_done / dt, 'unit': 'clips/s', 'cores': threads, 'kind': 'port',
            'sample': f'{n_done} x 1.5 s synthetic clips, batch 1: numpy python_speech_features-0.6 '
                      f'restatement + numpy float32 SI-NET (BLAS threads={threads})'}, \
        err_feat, err_prob


def main():
    args = parse()
    world, rank, local = dist_setup()
    from mmla_audio_amd import _lib, weights
    from mmla_audio_amd.synthetic import make_clips

    ctx = _lib.Context(local)
    if args.microbatch:
        ctx.set_microbatch(args.microbatch if args.workload == 'od_pipeline' else 0,
                           args.microbatch if args.workload == 'si_pipeline' else 0)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)
    wl = args.workload
    if wl == 'od_features':
        clips = args.clips or 4096
        clip_len = 40000
    elif wl == 'noise_gate':
        clips = args.clips or 4096
        clip_len = 40000
    elif wl == 'si_pipeline':
        clips = args.clips or 65536
        clip_len = 24000
    else:
        clips = args.clips or 65536
        clip_len = 40000

    W_od = weights.synthetic(weights.OD, seed=0)
    W_si = weights.synthetic(weights.SI, seed=0, n_classes=630)
    if wl == 'od_pipeline':
        ctx.load_weights(weights.OD, weights.pack(weights.OD, W_od), 2)
    if wl == 'si_pipeline':
        ctx.load_weights(weights.SI, weights.pack(weights.SI, W_si, 630), 630, _lib.HEAD_SOFTMAX)

    pcm = make_clips(clips, clip_len, start_index=rank * clips)
    if wl == 'noise_gate':   # float32 audio as librosa.load gives it, and a 10 s ambient-noise clip
        yf = (pcm.float() / 32768.0).contiguous()
        del pcm
        pcm = None
        gen = torch.Generator(device='cuda')
        gen.manual_seed(4242)
        noise_clip = (0.01 * torch.randn(160000, generator=gen, device='cuda')).cpu().numpy()
        ctx.nr_set_noise(noise_clip)
        nr_out = torch.empty_like(yf)
    K = 2 if wl == 'od_pipeline' else 630
    probs = torch.empty((clips, K), dtype=torch.float32, device='cuda')
    argmax = torch.empty(clips, dtype=torch.int32, device='cuda')
    norm = torch.empty((clips, 128, 151), dtype=torch.float32, device='cuda') if wl == 'od_features' else None
    zcr = torch.empty((clips, 151), dtype=torch.float32, device='cuda') if wl == 'od_features' else None
    gathered = torch.empty((world * clips, K), dtype=torch.float32, device='cuda') if world > 1 else None

    def step():
        if wl == 'od_pipeline':
            ctx.od_pipeline_dev(pcm.data_ptr(), clips, clip_len, clip_len, probs.data_ptr(),
                                argmax.data_ptr())
        elif wl == 'si_pipeline':
            ctx.si_pipeline_dev(pcm.data_ptr(), clips, clip_len, clip_len, probs.data_ptr(),
                                argmax.data_ptr())
        elif wl == 'noise_gate':
            ctx.nr_reduce_dev(yf.data_ptr(), clips, clip_len, clip_len, nr_out.data_ptr())
        else:
            ctx.od_features_dev(pcm.data_ptr(), clips, clip_len, clip_len, norm=norm.data_ptr(),
                                zcr=zcr.data_ptr())
        if world > 1 and wl not in ('od_features', 'noise_gate'):
            import torch.distributed as dist
            dist.all_gather_into_tensor(gathered, probs)   # RCCL over xGMI: logits to every rank

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.profile_read(reset=True)
    ctx.profile_enable(True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    ctx.profile_enable(False)
    prof = ctx.profile_read(reset=True)
    dt = max_over_ranks(dt, world)
    value = world * clips * args.steps / dt

    # dominant kernel and its roofline (algorithmic work / device time from HIP events)
    stage = max(prof, key=lambda s: prof[s][0])
    ms, launches, work = prof[stage]
    if stage in ('od_fe', 'si_fe', 'nr'):
        achieved = work / (ms * 1e-3) / 1e9
        roof = {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': achieved / HBM_PEAK_GBS, 'traffic': None}
    else:
        achieved = work / (ms * 1e-3) / 1e12
        peak = F16X3_PEAK_TFS if stage == 'conv' else F32_MFMA_PEAK_TFS
        roof = {'bound': 'mfma', 'achieved': achieved, 'peak': peak, 'unit': 'TFLOP/s',
                'frac': achieved / peak, 'traffic': None,
                'arith': '3xFP16 on f16 MFMA (peak = f16 dense / 3)' if stage == 'conv' else 'f32 MFMA'}
    roof.update({'kernel': stage, 'launches': launches, 'avg_launch_ms': ms / max(launches, 1),
                 'work_per_launch': work / max(launches, 1)})
    roof['traffic'], roof['traffic_source'] = pmc_traffic(wl, stage, clips)
    stages = {s: {'ms': round(v[0], 3), 'launches': v[1],
                  ('GB/s' if s in ('od_fe', 'si_fe', 'nr') else 'TFLOP/s'):
                      round(v[2] / (v[0] * 1e-3) / (1e9 if s in ('od_fe', 'si_fe', 'nr') else 1e12), 3)
                      if v[0] > 0 else 0.0}
              for s, v in prof.items() if v[1]}

    # front-end roofline on the same clips (config 2 measurement) for the pipeline workloads
    fe = None
    if wl == 'od_pipeline' and rank == 0:
        n_fe = min(clips, 4096)
        nrm = torch.empty((n_fe, 128, 151), dtype=torch.float32, device='cuda')
        zc = torch.empty((n_fe, 151), dtype=torch.float32, device='cuda')
        ctx.od_features_dev(pcm.data_ptr(), n_fe, clip_len, clip_len, norm=nrm.data_ptr(),
                            zcr=zc.data_ptr())
        torch.cuda.synchronize()
        ctx.profile_enable(True)
        for _ in range(3):
            ctx.od_features_dev(pcm.data_ptr(), n_fe, clip_len, clip_len, norm=nrm.data_ptr(),
                                zcr=zc.data_ptr())
        torch.cuda.synchronize()
        ctx.profile_enable(False)
        p = ctx.profile_read(reset=True)['od_fe']
        gbs = p[2] / (p[0] * 1e-3) / 1e9
        fe = {'kernel': 'od_fe', 'clips': n_fe, 'clips_per_s': n_fe * p[1] / (p[0] * 1e-3),
              'roofline': {'bound': 'hbm', 'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                           'frac': gbs / HBM_PEAK_GBS, 'traffic': None,
                           'avg_launch_ms': p[0] / max(p[1], 1), 'bytes_per_clip': OD_FE_BYTES}}

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        n_s = 64
        sample = pcm[:n_s].cpu().numpy() if pcm is not None else None
        if wl == 'noise_gate':
            cpu, e1 = cpu_baseline_nr(yf[:n_s].cpu().numpy(), noise_clip, nr_out[:n_s].cpu().numpy(),
                                      args.cpu_seconds)
            parity = {'nr_max_abs_err_vs_oracle': e1}
        elif wl == 'si_pipeline':
            feat = torch.empty((n_s, 256, 39), dtype=torch.float32, device='cuda')
            ctx.si_features_dev(pcm.data_ptr(), n_s, clip_len, clip_len, feat.data_ptr())
            torch.cuda.synchronize()
            cpu, e1, e2 = cpu_baseline_si(sample, feat.cpu().numpy(), probs[:n_s].cpu().numpy(),
                                          W_si, args.cpu_seconds)
            parity = {'si_feature_max_abs_err': e1, 'prob_max_abs_err': e2}
        else:
            nrm = torch.empty((n_s, 128, 151), dtype=torch.float32, device='cuda')
            ctx.od_features_dev(pcm.data_ptr(), n_s, clip_len, clip_len, norm=nrm.data_ptr())
            torch.cuda.synchronize()
            gp = probs[:n_s].cpu().numpy() if wl == 'od_pipeline' else np.zeros((n_s, 2))
            cpu, e1, e2 = cpu_baseline_od(sample, nrm.cpu().numpy(), gp, W_od, args.cpu_seconds)
            parity = {'od_norm_logmel_max_abs_err': e1}
            if wl == 'od_pipeline':
                parity['prob_max_abs_err'] = e2

    if rank == 0:
        desc = {
            'od_pipeline': 'config 3: fused log-mel/ZCR front-end -> uint8 image -> OD-NET ResLSTM '
                           '-> softmax, per GPU',
            'si_pipeline': 'config 4: MFCC+d+dd (float64) -> SI-NET Conv1D ResNet+BiLSTM -> '
                           'Dense(630) softmax, per GPU',
            'od_features': 'config 2: OD front-end kernel only (log-mel norm + ZCR out)',
            'noise_gate': 'SURVEY 8f row 3: nr.reduce_noise(stationary=True) gate on 2.5 s clips '
                          '(noisereduce 2.0 defaults, float64 STFT), per GPU',
        }[wl]
        line = {
            'metric': METRIC, 'value': value, 'unit': 'clips/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': dt / args.steps * 1e3,
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            # convolutions: error-compensated 3xFP16 on f16 MFMA with f32 accumulation; front-ends
            # f32 (OD) / f64 (SI); LSTM, heads f32
            'dtype': {'od_pipeline': 'f16x3+f32', 'si_pipeline': 'f64+f16x3',
                      'noise_gate': 'f64'}.get(wl, 'f32'),
            'data': (f'synthetic: {clips} x {clip_len / 16000:g} s 16 kHz clips per GPU generated in '
                     f'HBM (5 classes, SURVEY 8d)' +
                     (', as float32 audio, gated against a 10 s synthetic noise profile'
                      if wl == 'noise_gate' else
                      ' (int16); seeded synthetic weights in the reference variables.index layout '
                      '(trained blobs absent)')),
            'config': {'workload': f'{wl} ({desc})', 'clips_per_gpu': clips,
                       'global_batch': world * clips, 'clip_samples': clip_len,
                       'parallelism': f'dp{world}' + ('+rccl_allgather_logits' if world > 1 else '')},
            'roofline': roof, 'stages': stages, 'fe': fe, 'cpu_baseline': cpu, 'parity': parity,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
