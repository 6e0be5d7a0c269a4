"""3xFP16 range guard (include/mmla.h mmla_range_check).

The default arithmetic splits every conv / LSTM operand into fp16 hi + lo; a value >= 65504 would
become inf and could be masked downstream (ELU(-inf) = -1, MaxPool, LSTM saturation) into a finite,
wrong class.  Weights are split at a per-tensor power-of-two scale (any finite tensor fits; a
non-finite one makes the model run exact f32 at load time); activations outside the range are flagged by the kernel that splits them: host-pointer calls re-run the micro-batch in
exact f32 (bit-identical to MMLA_PREC_F32), device-pointer calls report MMLA_E_RANGE.
"""
import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu


def _ctx(W_od=None, W_si=None, prec=None):
    from mmla_audio_amd import _lib, weights
    c = _lib.Context(0)
    if W_od is not None:
        c.load_weights(weights.OD, weights.pack(weights.OD, W_od), 2)
    if W_si is not None:
        c.load_weights(weights.SI, weights.pack(weights.SI, W_si, 8), 8, _lib.HEAD_SIGMOID)
    if prec is not None:
        c.set_precision(prec)
    return c


def _hot_od():
    """OD weights whose block-4 BatchNorm drives its conv input past 65504 (lww-14 = block 4 BN1)."""
    from mmla_audio_amd import weights
    W = weights.synthetic(weights.OD, seed=5)
    W['layer_with_weights-14/gamma'] = W['layer_with_weights-14/gamma'] * 2.0e5
    W['layer_with_weights-14/beta'] = np.abs(W['layer_with_weights-14/beta']) * 2.0e5
    return W


def test_in_range_weights_report_nothing():
    from mmla_audio_amd import weights
    c = _ctx(W_od=weights.synthetic(weights.OD, seed=5))
    c.od_pipeline(synth.batch(300, 8, 40000))
    assert c.range_check() == 0


def test_od_activation_overflow_host_call_reruns_in_f32():
    from mmla_audio_amd import _lib
    W = _hot_od()
    pcm = synth.batch(310, 12, 40000)
    c = _ctx(W_od=W)
    p, a, _ = c.od_pipeline(pcm)
    assert c.range_check() >= 1                   # the micro-batch was re-run
    ref = _ctx(W_od=W, prec=_lib.PREC_F32)
    p32, a32, _ = ref.od_pipeline(pcm)
    assert np.all(np.isfinite(p))
    assert np.array_equal(p, p32) and np.array_equal(a, a32)


def test_od_activation_overflow_device_call_reports_range():
    import torch
    from mmla_audio_amd import _lib
    c = _ctx(W_od=_hot_od())
    pcm = torch.from_numpy(synth.batch(320, 4, 40000)).cuda()
    probs = torch.empty((4, 2), dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    c.od_pipeline_dev(pcm.data_ptr(), 4, 40000, 40000, probs.data_ptr())
    with pytest.raises(_lib.MmlaError) as e:
        c.range_check()
    assert e.value.code == _lib.MMLA_E_RANGE
    assert c.range_check() == 0                   # reported once, then cleared


def test_nonfinite_weights_run_exact_f32():
    """a weight tensor holding inf / NaN cannot be split: that model runs exact f32 (load time)"""
    from mmla_audio_amd import _lib, weights
    W = weights.synthetic(weights.OD, seed=6)
    W['layer_with_weights-20/kernel'] = W['layer_with_weights-20/kernel'].copy()
    W['layer_with_weights-20/kernel'][0, 0, 0, 0] = np.inf      # block 5's 3x3 conv
    pcm = synth.batch(330, 6, 40000)
    c = _ctx(W_od=W)
    p, a, _ = c.od_pipeline(pcm)
    ref = _ctx(W_od=W, prec=_lib.PREC_F32)
    p32, a32, _ = ref.od_pipeline(pcm)
    assert np.array_equal(p, p32, equal_nan=True) and np.array_equal(a, a32)
    assert c.range_check() == 0                   # decided at load time, nothing re-run


def _scaled_od(f, seed=16):
    """OD weights with every 3x3 conv kernel and bias x f (its BatchNorm's moving mean x f and
    variance x f^2, so the block still sees O(1) activations) and the BiLSTM kernels x f"""
    from mmla_audio_amd import weights
    W = weights.synthetic(weights.OD, seed=seed)
    names = [e[0] for e in weights.spec(weights.OD)]
    for i, name in enumerate(names):
        if name.endswith('/kernel') and W[name].ndim == 4 and W[name].shape[:2] == (3, 3):
            W[name] = W[name] * f
            W[name.replace('/kernel', '/bias')] = W[name.replace('/kernel', '/bias')] * f
            bn = next(m for m in names[i:] if m.endswith('/moving_variance'))
            W[bn] = W[bn] * f * f
            W[bn.replace('moving_variance', 'moving_mean')] = W[bn.replace('moving_variance', 'moving_mean')] * f
        if 'layer_with_weights-40/' in name and name.endswith('kernel'):
            W[name] = W[name] * f
    return W


@pytest.mark.parametrize('f', [1.0e4, 1.0e-3])
def test_scaled_weights_stay_on_3xfp16(f):
    """each weight tensor is split at its own power-of-two scale, so weights far
    outside the old fixed 2^8 window (|w| up to ~1.5e3 here, or ~1e-4) keep the 3xFP16 path:
    log-probabilities within 1e-4 of the float64 oracle, nothing flagged, no exact-f32 fallback"""
    from mmla_audio_amd import _lib
    from oracle import compare, nets
    W = _scaled_od(f)
    m = [float(np.abs(W[k]).max()) for k in W if k.endswith('kernel')]
    assert max(m) > 255.9 if f > 1 else min(m) < 1e-3        # outside the old fixed 2^8 window
    x = np.random.default_rng(17).integers(0, 256, size=(6, 128, 151, 3)).astype(np.uint8)
    c = _ctx(W_od=W)
    p = c.od_forward(x)
    assert c.range_check() == 0
    ref = nets.od_forward(x.astype(np.float32), W)
    assert compare.logp_err(p, ref) <= compare.LOGP_TOL, compare.logp_err(p, ref)
    assert compare.argmax_ok(p, ref)
    p32 = _ctx(W_od=W, prec=_lib.PREC_F32).od_forward(x)
    assert not np.array_equal(p, p32)             # really the 3xFP16 arithmetic, not the f32 path


def test_si_lstm_input_overflow_host_call_reruns_in_f32():
    from mmla_audio_amd import _lib, weights
    W = weights.synthetic(weights.SI, seed=7, n_classes=8)
    # final BN (lww-40) feeds ReLU -> AvgPool -> BiLSTM input: |x| > 1023 overflows x * 2^6
    W['layer_with_weights-40/gamma'] = W['layer_with_weights-40/gamma'] * 1.0e4
    W['layer_with_weights-40/beta'] = np.abs(W['layer_with_weights-40/beta']) * 1.0e4
    pcm = synth.batch(340, 10, 24000)
    c = _ctx(W_si=W)
    p, a, _ = c.si_pipeline(pcm)
    assert c.range_check() >= 1
    ref = _ctx(W_si=W, prec=_lib.PREC_F32)
    p32, a32, _ = ref.si_pipeline(pcm)
    assert np.array_equal(p, p32) and np.array_equal(a, a32)


def test_float_pcm_outside_split_range():
    """the float-PCM front-end splits y 2^3 into fp16, so |y| must stay below 8188.
    A host call with a larger (or non-finite) sample in the 24 000-sample window returns MMLA_E_RANGE
    instead of an overflowed image; one outside the window is never read and passes; a device-pointer
    call reports it from mmla_synchronize.  In-range loud float audio (|y| up to 8000) is exact."""
    import torch
    from mmla_audio_amd import _lib
    c = _ctx()
    y = (synth.clip(7, 30000).astype(np.float32) / 32768.0)
    loud = y * 8000.0 / np.abs(y).max()
    f = c.od_features(loud[None])
    assert np.isfinite(f['db']).all()
    bad = loud.copy()
    bad[1234] = 9000.0
    with pytest.raises(_lib.MmlaError) as e:
        c.od_features(bad[None])
    assert e.value.code == _lib.MMLA_E_RANGE
    assert 'clip 0 sample 1234' in str(e.value)
    # the kernel's range word flags the host call; the host re-scan names the clip of a batch
    with pytest.raises(_lib.MmlaError) as e:
        c.od_features(np.stack([loud, loud, bad]))
    assert e.value.code == _lib.MMLA_E_RANGE and 'clip 2 sample 1234' in str(e.value)
    assert np.isfinite(c.od_features(np.stack([loud, loud]))['db']).all()   # the word was reset
    nan = loud.copy()
    nan[10] = np.nan
    with pytest.raises(_lib.MmlaError):
        c.od_features(nan[None])
    late = loud.copy()
    late[25000] = 9000.0           # past the 24 000 samples the front-end reads
    c.od_features(late[None])
    dev = torch.from_numpy(bad[None]).cuda()
    out = torch.empty((1, 128, 151), dtype=torch.float32, device='cuda')
    c.set_stream(torch.cuda.current_stream().cuda_stream)
    c._check(c.lib.mmla_od_features_f32(c.h, dev.data_ptr(), 1, 30000, None, 30000, None, out.data_ptr(),
                                        None, None, _lib.MMLA_DEVICE_PTR), 'f32 dev')
    with pytest.raises(_lib.MmlaError) as e:
        c.synchronize()
    assert e.value.code == _lib.MMLA_E_RANGE
    c.synchronize()


@pytest.mark.parametrize('bn', [3, 6, 12, 36])
def test_si_chain_overflow_host_call_reruns_in_f32(bn):
    """every split inside the fused SI res-unit chains (siu.hip siu_chain_kernel) is range-guarded:
    a BatchNorm scaled past the fp16 range in the pool unit's t1 (lww-3), the second unit's input
    (lww-6), the third unit's t1 (lww-12) or the last chain's unit 9 input (lww-36) flags the launch,
    and the host call re-runs the micro-batch in exact f32"""
    from mmla_audio_amd import _lib, weights
    W = weights.synthetic(weights.SI, seed=8, n_classes=8)
    W[f'layer_with_weights-{bn}/gamma'] = W[f'layer_with_weights-{bn}/gamma'] * 1.0e5
    W[f'layer_with_weights-{bn}/beta'] = np.abs(W[f'layer_with_weights-{bn}/beta']) * 1.0e5
    pcm = synth.batch(350 + bn, 6, 24000)
    c = _ctx(W_si=W)
    p, a, _ = c.si_pipeline(pcm)
    assert c.range_check() >= 1
    p32, a32, _ = _ctx(W_si=W, prec=_lib.PREC_F32).si_pipeline(pcm)
    assert np.array_equal(p, p32) and np.array_equal(a, a32)
