"""3xFP16 range guard (include/mmla.h mmla_range_check).

The default arithmetic splits every conv / LSTM operand into fp16 hi + lo; a value >= 65504 would
become inf and could be masked downstream (ELU(-inf) = -1, MaxPool, LSTM saturation) into a finite,
wrong class.  Weights outside the range make the model run exact f32 at load time; activations
outside it are flagged by the kernel that splits them: host-pointer calls re-run the micro-batch in
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


@pytest.mark.parametrize('big', [300.0, 7.0e4])
def test_out_of_range_weights_run_exact_f32(big):
    """conv_h3 splits w * 2^8: |w| >= 65504 / 2^8 (= 255.9) already leaves the fp16 range"""
    from mmla_audio_amd import _lib, weights
    W = weights.synthetic(weights.OD, seed=6)
    W['layer_with_weights-20/kernel'] = W['layer_with_weights-20/kernel'].copy()
    W['layer_with_weights-20/kernel'][0, 0, 0, 0] = big      # block 5's 3x3 conv
    pcm = synth.batch(330, 6, 40000)
    c = _ctx(W_od=W)
    p, a, _ = c.od_pipeline(pcm)
    ref = _ctx(W_od=W, prec=_lib.PREC_F32)
    p32, a32, _ = ref.od_pipeline(pcm)
    assert np.array_equal(p, p32) and np.array_equal(a, a32)
    assert c.range_check() == 0                   # decided at load time, nothing re-run


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
