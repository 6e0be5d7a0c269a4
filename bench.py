#!/usr/bin/env python3
"""Benchmark: audio clips/s (MFCC -> logits) on 1..8 MI355X, one process per GPU.

  python bench.py [--gpus N --steps K --warmup W --workload od_pipeline|si_pipeline|od_features|noise_gate]

With --gpus N > 1 and no torchrun environment, bench.py starts
`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py` as a child
process before anything touches a GPU and exits with its code; under torchrun (WORLD_SIZE set) each
rank drives its LOCAL_RANK GPU and the per-step probabilities are all-gathered over RCCL.

A step = one pass of the hot path over one batch of synthetic clips already resident in HBM:
  od_pipeline (default, BASELINE config 3): 65 536 x 2.5 s clips / GPU, fused log-mel+ZCR front-end
      -> quantised image -> OD-NET (Conv2D ResNet + BiLSTM + Dense) -> softmax/argmax;
      at N GPUs the per-shard probabilities are all-gathered over RCCL (config 5 at N = 8).
  si_pipeline (config 4): 65 536 x 1.5 s clips / GPU, MFCC+delta+delta-delta -> SI-NET, K = 630.
  od_features (config 2): the front-end kernel alone, 4 096 x 2.5 s clips / GPU.
  noise_gate: the stationary noise gate on 4 096 x 2.5 s clips / GPU.
Prints ONE JSON line (rank 0) with roofline + cpu_baseline objects.
"""
import argparse
import json
import os
import socket
import subprocess
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
HBM_STAGES = ('od_fe', 'si_fe', 'nr')
PREC_F32, PREC_F16X3 = 0, 1


def pmc_traffic(workload, stage, clips_per_launch):
    """HBM bytes per launch of `stage` from the committed PMC capture of this workload
    (tools/gpu/pmc_traffic.sh -> profiles/pmc_traffic_<workload>.json), scaled to this run's clips
    per launch; None when no capture exists."""
    path = os.path.join(REPO, 'profiles', f'pmc_traffic_{workload}.json')
    try:
        d = json.load(open(path))
        st = d['stages'][stage]
        per_clip = st['traffic_bytes_per_launch'] / d['clips_per_launch'][stage]
        return per_clip * clips_per_launch, os.path.relpath(path, REPO)
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=None,
                    help='timed steps (default 3; 50 for od_features, whose step is one ~0.3 ms '
                         'launch, so that host-side jitter stays out of the value)')
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--workload', default='od_pipeline',
                    choices=['od_pipeline', 'si_pipeline', 'od_features', 'noise_gate'])
    ap.add_argument('--clips', type=int, default=None, help='clips per GPU')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-f32', action='store_true', help='skip the exact-f32 precision leg')
    ap.add_argument('--no-parity', action='store_true', help='skip the oracle parity sample')
    ap.add_argument('--no-latency', action='store_true', help='skip the batch-1 latency probe')
    ap.add_argument('--microbatch', type=int, default=0,
                    help='clips per internal micro-batch (0 = the library default)')
    ap.add_argument('--cpu-seconds', type=float, default=20.0)
    ap.add_argument('--classes', type=int, default=630,
                    help='si_pipeline: speakers K of the Dense head (630 = the base model; SURVEY 8(d) '
                         'config 4 also asks for K = 8 with the deployed sigmoid head)')
    ap.add_argument('--head', choices=['softmax', 'sigmoid'], default=None,
                    help='si_pipeline head (default: softmax for K = 630, sigmoid otherwise -- '
                         'transfer_learning\'s customized_dense, speaker_identification.py:409)')
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 50 if args.workload == 'od_features' else 3
    if args.head is None:
        args.head = 'softmax' if args.classes == 630 else 'sigmoid'
    return args


def launch_ranks(args):
    """--gpus N outside torchrun: run N ranks under torch.distributed.run as a child process
    (no GPU has been touched in this process) and return its exit code."""
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           f'--nproc-per-node={args.gpus}', '--master-addr', '127.0.0.1', '--master-port', str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR='127.0.0.1'))


def dist_setup():
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
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


def rank_devices(world, rank, local):
    p = torch.cuda.get_device_properties(local)
    me = {'rank': rank, 'local_rank': local, 'device': local, 'name': p.name,
          'pci_bus_id': getattr(p, 'pci_bus_id', None), 'pci_device_id': getattr(p, 'pci_device_id', None),
          'host': socket.gethostname()}
    if world == 1:
        return [me]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, me)
    return out


def roofline(prof, wl, clips_per_launch, prec, stage=None):
    """dominant stage (or `stage`): algorithmic work per launch / average launch time (HIP events)"""
    if stage is None:
        stage = max(prof, key=lambda s: prof[s][0])
    ms, launches, work = prof[stage]
    if stage in HBM_STAGES:
        achieved = work / (ms * 1e-3) / 1e9
        roof = {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': achieved / HBM_PEAK_GBS, 'traffic': None}
    else:
        achieved = work / (ms * 1e-3) / 1e12
        f16 = stage in ('conv', 'lstm') and prec == PREC_F16X3
        peak = F16X3_PEAK_TFS if f16 else F32_MFMA_PEAK_TFS
        roof = {'bound': 'mfma', 'achieved': achieved, 'peak': peak, 'unit': 'TFLOP/s',
                'frac': achieved / peak, 'traffic': None,
                'arith': '3xFP16 on f16 MFMA (peak = f16 dense / 3)' if f16 else 'f32 MFMA'}
    roof.update({'kernel': stage, 'launches': launches, 'avg_launch_ms': ms / max(launches, 1),
                 'work_per_launch': work / max(launches, 1)})
    roof['traffic'], roof['traffic_source'] = pmc_traffic(wl, stage, clips_per_launch)
    return roof


def stage_table(prof):
    return {s: {'ms': round(v[0], 3), 'launches': v[1],
                ('GB/s' if s in HBM_STAGES else 'TFLOP/s'):
                    round(v[2] / (v[0] * 1e-3) / (1e9 if s in HBM_STAGES else 1e12), 3) if v[0] > 0 else 0.0}
            for s, v in prof.items() if v[1]}


def sample_indices(n, mb, k, seed=20261015):
    """first and last clip of every micro-batch + k seeded random clips"""
    idx = set()
    for c0 in range(0, n, mb):
        idx.update((c0, min(c0 + mb, n) - 1))
    idx.update(np.random.default_rng(seed).choice(n, min(k, n), replace=False).tolist())
    return sorted(idx)


def fe_sample_indices(n, grid, k=24, seed=20261015):
    """od_features: clips the persistent front-end's workgroups run first, in the middle and last
    (workgroup b owns clips b, b + grid, ...) + k seeded random clips"""
    idx = {0, n - 1}
    for b in (0, grid // 3, grid // 2, grid - 1):
        owned = list(range(b, n, grid))
        if owned:
            idx.update((owned[0], owned[len(owned) // 2], owned[-1]))
    idx.update(np.random.default_rng(seed).choice(n, min(k, n), replace=False).tolist())
    return sorted(i for i in idx if 0 <= i < n)


def parity_sample(ctx, wl, pcm, probs, argmax, W, mb, clip_len, k=24, fe_out=None, head='softmax'):
    """oracle (float64) vs the timed run's outputs on clips spread across the whole batch"""
    from oracle import od_fe, si_fe
    from oracle.nets_torch import Nets
    n = pcm.shape[0]
    if wl == 'od_features':
        grid = min(n, torch.cuda.get_device_properties(pcm.device).multi_processor_count)
        idx = fe_sample_indices(n, grid, k)
    else:
        idx = sample_indices(n, mb, k)
    sub = pcm[idx].contiguous()
    host = sub.cpu().numpy()
    out = {'sample_clips': len(idx), 'sample': 'first + last clip of every micro-batch and '
           f'{min(k, n)} seeded random clips of the {n}-clip batch; float64 oracle'}
    if wl == 'od_features':
        # the TIMED run's own outputs (the last timed step wrote norm / zcr), at clips that the
        # persistent workgroups process first, in the middle and last
        out['sample'] = (f'the timed launch\'s norm / zcr outputs of {len(idx)} clips: first / middle / '
                         f'last clip of 4 of the {grid} persistent workgroups + {min(k, n)} seeded '
                         'random clips; float64 oracle')
        norm = fe_out[0][idx].cpu().numpy()
        zc = fe_out[1][idx].cpu().numpy()
    elif wl == 'od_pipeline':
        nrm = torch.empty((len(idx), 128, 151), dtype=torch.float32, device='cuda')
        gim = torch.empty((len(idx), 128, 151, 3), dtype=torch.uint8, device='cuda')
        ctx.od_features_dev(sub.data_ptr(), len(idx), clip_len, clip_len, norm=nrm.data_ptr())
        # the image the pipeline's network reads (the fused pipeline = od_forward_u8 on it, bit for bit)
        ctx.od_features_dev(sub.data_ptr(), len(idx), clip_len, clip_len, img=gim.data_ptr())
        torch.cuda.synchronize()
        norm = nrm.cpu().numpy()
        gimg = gim.cpu().numpy()
        zc = None
    if wl in ('od_pipeline', 'od_features'):
        feats = [od_fe.od_features(host[j]) for j in range(len(idx))]
        err = 0.0
        zbad = 0
        for j, f in enumerate(feats):
            ok = ~np.isnan(f['norm'])
            if ok.any():
                err = max(err, float(np.abs(norm[j][ok] - f['norm'][ok]).max()))
            if zc is not None:
                zbad += int(not np.array_equal(np.rint(zc[j] * 400).astype(int),
                                               np.rint(f['zcr'][0] * 400).astype(int)))
        out['od_norm_logmel_max_abs_err'] = err
        if zc is not None:
            out['zcr_count_mismatch_clips'] = zbad
        if wl == 'od_pipeline':
            oimg = np.stack([f['png_rgb'] for f in feats])
            net = Nets(W)
            ref = net.od_forward(oimg.astype(np.float32))
            # the network alone: the oracle net on the GPU's OWN image (the
            # end-to-end figure also carries the image's permitted 1-LSB pixel values, which the
            # seeded net amplifies)
            ref_net = net.od_forward(gimg.astype(np.float32))
            lsb = np.abs(gimg.astype(np.int16) - oimg.astype(np.int16))
            out['img_lsb_pixels'] = int((lsb > 0).sum())
            out['img_pixel_values'] = int(lsb.size)
            out['img_max_lsb'] = int(lsb.max())
    else:
        feat = torch.empty((len(idx), 256, 39), dtype=torch.float32, device='cuda')
        ctx.si_features_dev(sub.data_ptr(), len(idx), clip_len, clip_len, feat.data_ptr())
        torch.cuda.synchronize()
        xs = np.stack([si_fe.input_feature_gen(host[j])[0] for j in range(len(idx))])
        out['si_feature_max_abs_err'] = float(np.abs(feat.cpu().numpy() - xs).max())
        ref = Nets(W).si_forward(xs.astype(np.float32), head=head)
    if wl in ('od_pipeline', 'si_pipeline'):
        from oracle import compare
        gp = probs[idx].cpu().numpy()
        ga = argmax[idx].cpu().numpy()
        agree, disagree, ties = compare.argmax_report(gp, ref)
        if wl == 'od_pipeline':
            with np.errstate(divide='ignore'):
                e2e = np.abs(np.log(gp.astype(np.float64)) - np.log(ref)).max(1)
                own = np.abs(np.log(gp.astype(np.float64)) - np.log(ref_net)).max(1)
            j = int(e2e.argmax())
            out.update({'logp_err_net': compare.logp_err(gp, ref_net),
                        'logp_err_net_bar': compare.LOGP_TOL,
                        'worst_clip': {'index': int(idx[j]), 'logp_err_e2e': float(e2e[j]),
                                       'logp_err_net': float(own[j]),
                                       'img_lsb_pixels': int((lsb[j] > 0).sum())},
                        'logp_err_note': 'logp_max_abs_err = GPU pipeline vs the oracle net on the '
                                         'ORACLE image (includes 1-LSB image differences); '
                                         'logp_err_net = vs the oracle net on the GPU image'})
        out.update({'logp_max_abs_err': compare.logp_err(gp, ref), 'prob_max_abs_err': float(np.abs(gp - ref).max()),
                    'argmax_agree': agree, 'argmax_disagree_non_tie': disagree,
                    'argmax_matches_probs': bool(np.array_equal(ga, gp.argmax(1))),
                    'near_ties_log_margin': ties, 'tie_rule': f'top-2 log-margin < {compare.TIE_LOG_MARGIN:g}'})
    return out


def main():
    args = parse()
    world_env = int(os.environ.get('WORLD_SIZE', '1'))
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch_ranks(args))
    if world_env != args.gpus:
        print(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}: measuring {world_env} '
              'rank(s)', file=sys.stderr)
    rank = int(os.environ.get('RANK', '0'))
    wl = args.workload

    # CPU baseline first, before this process touches a GPU (child processes, pinned cores)
    cpu = None
    if rank == 0 and world_env == 1 and not args.no_cpu_baseline:
        from oracle import cpu_baseline
        cpu = cpu_baseline.run_modes(wl, args.cpu_seconds)

    world, rank, local = dist_setup()
    from mmla_audio_amd import _lib, weights
    from mmla_audio_amd.distributed import gather_logits
    from mmla_audio_amd.synthetic import make_clips

    ctx = _lib.Context(local)
    if args.microbatch:
        ctx.set_microbatch(args.microbatch if wl == 'od_pipeline' else 0,
                           args.microbatch if wl == 'si_pipeline' else 0)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)
    clips = args.clips or (65536 if wl in ('od_pipeline', 'si_pipeline') else 4096)
    clip_len = 24000 if wl == 'si_pipeline' else 40000

    W = None
    if wl == 'od_pipeline':
        W = weights.synthetic(weights.OD, seed=0)
        ctx.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    if wl == 'si_pipeline':
        W = weights.synthetic(weights.SI, seed=0, n_classes=args.classes)
        ctx.load_weights(weights.SI, weights.pack(weights.SI, W, args.classes), args.classes,
                         _lib.HEAD_SOFTMAX if args.head == 'softmax' else _lib.HEAD_SIGMOID)
    mb_od, mb_si = ctx.get_microbatch()
    mb = {'od_pipeline': mb_od, 'si_pipeline': mb_si}.get(wl, clips)

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
    K = 2 if wl == 'od_pipeline' else args.classes
    probs = torch.empty((clips, K), dtype=torch.float32, device='cuda')
    argmax = torch.empty(clips, dtype=torch.int32, device='cuda')
    norm = torch.empty((clips, 128, 151), dtype=torch.float32, device='cuda') if wl == 'od_features' else None
    zcr = torch.empty((clips, 151), dtype=torch.float32, device='cuda') if wl == 'od_features' else None
    pipeline = wl in ('od_pipeline', 'si_pipeline')
    gathered = torch.empty((world * clips, K), dtype=torch.float32, device='cuda') if pipeline else None

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
        if pipeline and world > 1:   # every rank ends the step with the whole batch's probabilities
            gather_logits(probs, n_total=world * clips, out=gathered)

    def timed(steps, warmup):
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        ctx.profile_read(reset=True)
        ctx.profile_enable(True)
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        barrier(world)
        dt = time.perf_counter() - t0
        ctx.profile_enable(False)
        return max_over_ranks(dt, world), ctx.profile_read(reset=True)

    dt, prof = timed(args.steps, args.warmup)
    value = world * clips * args.steps / dt
    roof = roofline(prof, wl, mb, PREC_F16X3)
    # the convolution stack's own roofline when another stage dominates the step (the SI pipeline since
    # round 6: its float64 front-end takes longer than the fused res-unit chains)
    roof_conv = (roofline(prof, wl, mb, PREC_F16X3, 'conv')
                 if roof['kernel'] != 'conv' and prof.get('conv', (0, 0, 0))[1] else None)
    stages = stage_table(prof)
    range_ok = True
    try:
        ctx.range_check()
    except _lib.MmlaError:
        range_ok = False

    # the exact-f32 arithmetic on the same batch (N = 1): value and roofline beside the 3xFP16 one,
    # and how many argmax labels the two arithmetics disagree on
    f32 = None
    if pipeline and world == 1 and not args.no_f32:
        am16 = argmax.clone()
        ctx.set_precision(PREC_F32)
        steps32 = max(1, min(args.steps, 2))
        dt32, prof32 = timed(steps32, 1)
        ctx.set_precision(PREC_F16X3)
        f32 = {'value': clips * steps32 / dt32, 'ms_per_step': dt32 / steps32 * 1e3, 'steps': steps32,
               'dtype': 'f32' if wl == 'od_pipeline' else 'f64+f32',
               'roofline': roofline(prof32, wl + '_f32', mb, PREC_F32), 'stages': stage_table(prof32),
               'argmax_differs_from_f16x3': int((argmax != am16).sum().item())}
        step()   # leave the 3xFP16 outputs in probs / argmax for the parity sample
        torch.cuda.synchronize()

    # front-end roofline on the same clips (config 2 measurement) for the OD pipeline
    fe = None
    if wl == 'od_pipeline' and rank == 0:
        n_fe = min(clips, 4096)
        nrm = torch.empty((n_fe, 128, 151), dtype=torch.float32, device='cuda')
        zc = torch.empty((n_fe, 151), dtype=torch.float32, device='cuda')
        ctx.od_features_dev(pcm.data_ptr(), n_fe, clip_len, clip_len, norm=nrm.data_ptr(),
                            zcr=zc.data_ptr())
        torch.cuda.synchronize()
        ctx.profile_enable(True)
        # 20 launches of ~0.3 ms (as the od_features line's 50 steps: over 3 the first launches'
        # warm-up moved the average by ~7 %)
        for _ in range(20):
            ctx.od_features_dev(pcm.data_ptr(), n_fe, clip_len, clip_len, norm=nrm.data_ptr(),
                                zcr=zc.data_ptr())
        torch.cuda.synchronize()
        ctx.profile_enable(False)
        p = ctx.profile_read(reset=True)['od_fe']
        gbs = p[2] / (p[0] * 1e-3) / 1e9
        fe = {'kernel': 'od_fe', 'clips': n_fe, 'clips_per_s': n_fe * p[1] / (p[0] * 1e-3),
              'roofline': {'bound': 'hbm', 'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                           'frac': gbs / HBM_PEAK_GBS, 'avg_launch_ms': p[0] / max(p[1], 1),
                           'bytes_per_clip': OD_FE_BYTES}}
        fe['roofline']['traffic'], fe['roofline']['traffic_source'] = pmc_traffic('od_features', 'od_fe', n_fe)

    parity = None
    if rank == 0 and not args.no_parity:
        if wl == 'noise_gate':
            from oracle import noisereduce as onr
            idx = sample_indices(clips, clips, 6)[:8]
            err = 0.0
            for i in idx:
                w = onr.reduce_noise(yf[i].cpu().numpy(), 16000, noise_clip)
                err = max(err, float(np.abs(nr_out[i].cpu().numpy() - w).max()))
            parity = {'sample_clips': len(idx), 'nr_max_abs_err_vs_oracle': err}
        else:
            parity = parity_sample(ctx, wl, pcm, probs, argmax, W, mb, clip_len,
                                   fe_out=(norm, zcr) if wl == 'od_features' else None, head=args.head)

    # batch-1 latency of the host-pointer call the reference's real-time loop makes (one 2.56 s
    # window per predict, record_on_pc.py:139-160): median of 20 after 5 warmups, outside the
    # timed region; informational (the headline is the batched throughput above)
    latency = None
    if pipeline and world == 1 and not args.no_latency:
        one = np.ascontiguousarray(pcm[:1].cpu().numpy())
        call = ctx.od_pipeline if wl == 'od_pipeline' else ctx.si_pipeline
        ts = []
        for i in range(25):
            t0 = time.perf_counter()
            call(one)
            if i >= 5:
                ts.append(time.perf_counter() - t0)
        latency = {'batch1_ms_median': 1e3 * float(np.median(ts)), 'batch1_ms_p90':
                   1e3 * float(np.percentile(ts, 90)), 'call': f'{wl} host pointers, 1 clip'}

    devices = rank_devices(world, rank, local)
    if rank == 0:
        desc = {
            'od_pipeline': 'config 3: fused log-mel/ZCR front-end -> uint8 image -> OD-NET ResLSTM '
                           '-> softmax, per GPU',
            'si_pipeline': 'config 4: MFCC+d+dd (float64) -> SI-NET Conv1D ResNet+BiLSTM -> '
                           f'Dense({args.classes}) {args.head}, per GPU',
            'od_features': 'config 2: OD front-end kernel only (log-mel norm + ZCR out)',
            'noise_gate': 'SURVEY 8f row 3: nr.reduce_noise(stationary=True) gate on 2.5 s clips '
                          '(noisereduce 2.0 defaults, float64 STFT), per GPU',
        }[wl]
        line = {
            'metric': METRIC, 'value': value, 'unit': 'clips/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': dt / args.steps * 1e3,
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            # convolutions + LSTM: error-compensated 3xFP16 on f16 MFMA with f32 accumulation;
            # front-ends f32 (OD) / f64 (SI); heads f32.  The exact-f32 run is `precision_f32`.
            'dtype': {'od_pipeline': 'f16x3+f32', 'si_pipeline': 'f64+f16x3',
                      'noise_gate': 'f64'}.get(wl, 'f32'),
            'data': (f'synthetic: {clips} x {clip_len / 16000:g} s 16 kHz clips per GPU generated in '
                     f'HBM (5 classes, SURVEY 8d)' +
                     (', as float32 audio, gated against a 10 s synthetic noise profile'
                      if wl == 'noise_gate' else
                      ' (int16); seeded synthetic weights in the reference variables.index layout '
                      '(trained blobs absent)')),
            'config': {'workload': f'{wl} ({desc})', 'clips_per_gpu': clips,
                       **({'classes': args.classes, 'head': args.head} if wl == 'si_pipeline' else {}),
                       'global_batch': world * clips, 'clip_samples': clip_len, 'microbatch': mb,
                       'parallelism': f'dp{world}' + ('+rccl_allgather_logits' if world > 1 and pipeline else '')},
            'world_size': world, 'gpus_requested': args.gpus, 'rank_devices': devices,
            'roofline': roof, 'roofline_conv': roof_conv, 'stages': stages, 'fe': fe, 'precision_f32': f32,
            'range_guard_ok': range_ok, 'cpu_baseline': cpu, 'parity': parity,
            'latency': latency,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
