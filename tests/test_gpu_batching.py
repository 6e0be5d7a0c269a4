"""Batch composition must not change any clip's result (the reference runs batch 1 per clip).

Every kernel works per clip (the fused conv tiles never straddle clips), so a clip's outputs are
bit-identical whether it runs alone, inside a large batch, or across micro-batch boundaries.
"""
import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from mmla_audio_amd import _lib, weights
    c = _lib.Context(0)
    W = weights.synthetic(weights.OD, seed=21)
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    Ws = weights.synthetic(weights.SI, seed=22, n_classes=8)
    c.load_weights(weights.SI, weights.pack(weights.SI, Ws, 8), 8, 1)
    return c


def test_od_batch_invariance(ctx):
    pcm = synth.batch(800, 37, 40000)
    p_all, a_all, _ = ctx.od_pipeline(pcm)
    for i in (0, 17, 36):
        p1, a1, _ = ctx.od_pipeline(pcm[i:i + 1])
        assert np.array_equal(p1[0], p_all[i]) and a1[0] == a_all[i]


def test_od_microbatch_boundaries(ctx):
    pcm = synth.batch(900, 150, 40000)
    p_ref, a_ref, _ = ctx.od_pipeline(pcm)
    ctx.set_microbatch(64, 0)            # 150 clips -> 64 + 64 + 22
    try:
        p, a, _ = ctx.od_pipeline(pcm)
        f = ctx.od_features(pcm[:70], db=False, zcr=False)
        x = ctx.od_forward(f['img'])
    finally:
        ctx.set_microbatch(0, 0)   # back to the defaults
    assert np.array_equal(p, p_ref) and np.array_equal(a, a_ref)
    assert np.array_equal(x, p_ref[:70])


def test_si_microbatch_boundaries(ctx):
    lens = [24000 if i % 7 else 3000 for i in range(50)]
    pcm = [synth.clip(1000 + i, n) for i, n in enumerate(lens)]
    p_ref, a_ref, s_ref = ctx.si_pipeline(pcm)
    ctx.set_microbatch(0, 16)            # 50 clips -> 16 + 16 + 16 + 2
    try:
        p, a, s = ctx.si_pipeline(pcm)
    finally:
        ctx.set_microbatch(0, 0)   # back to the defaults
    assert np.array_equal(p, p_ref) and np.array_equal(a, a_ref) and np.array_equal(s, s_ref)


def test_empty_batches(ctx):
    p, a, _ = ctx.od_pipeline(np.zeros((0, 40000), np.int16))
    assert p.shape == (0, 2) and a.shape == (0,)
    f = ctx.od_features(np.zeros((0, 40000), np.int16))
    assert f['norm'].shape == (0, 128, 151)
    x = ctx.od_forward(np.zeros((0, 128, 151, 3), np.float32))
    assert x.shape == (0, 2)


def test_od_silent_gate(ctx):
    """record_on_pc.py:141-154: fewer than 4000 samples -> 'silent' (argmax -1), others classify
    exactly as they do alone."""
    lens = [3999, 4000, 40000, 0, 100, 23999]
    pcm = [synth.clip(1500 + i, n) for i, n in enumerate(lens)]
    p, a, s = ctx.od_pipeline(pcm)
    assert s.tolist() == [True, False, False, True, True, False]
    assert all(a[i] == -1 for i in (0, 3, 4))
    for i in (1, 2, 5):
        p1, a1, s1 = ctx.od_pipeline(pcm[i][None])
        assert not s1[0] and a1[0] == a[i] and np.array_equal(p1[0], p[i])
    # without lens the clip length decides for every clip
    _, a2, s2 = ctx.od_pipeline(np.zeros((3, 3000), np.int16))
    assert s2.all() and (a2 == -1).all()


def test_oom_retry_halves_this_call_only(monkeypatch):
    """a workspace OOM halves the micro-batch for the rest of that call and nothing
    else -- the next call is sized from free memory again (MMLA_DEBUG_FAIL_ALLOC=1 injects one
    allocation failure into a fresh context)."""
    from mmla_audio_amd import _lib, weights
    W = weights.synthetic(weights.OD, seed=21)
    pcm = synth.batch(950, 150, 40000)
    ref = _lib.Context(0)
    ref.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    p_ref, a_ref, _ = ref.od_pipeline(pcm)
    monkeypatch.setenv('MMLA_DEBUG_FAIL_ALLOC', '1')
    c = _lib.Context(0)
    monkeypatch.delenv('MMLA_DEBUG_FAIL_ALLOC')
    c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
    mb0 = c.get_microbatch()[0]
    assert mb0 >= 150
    p, a, _ = c.od_pipeline(pcm)        # first workspace allocation fails -> 75 + 75
    assert np.array_equal(p, p_ref) and np.array_equal(a, a_ref)
    assert c.get_microbatch()[0] == mb0  # not capped at 75 for later calls
    p2, _, _ = c.od_pipeline(pcm)
    assert np.array_equal(p2, p_ref)


def test_large_batches_match_batch_one(ctx):
    """Batches of >= 8192 clips run the BiLSTM with 64-clip workgroups (nets.hip LSTM_MT2_MIN), small
    ones with 32-clip workgroups: the same clip must give the same bits either way (OD and SI)."""
    base_od = synth.batch(1700, 24, 40000)
    pcm = np.tile(base_od, (342, 1))[:8200]          # 8200 clips, 24 distinct
    p_all, a_all, _ = ctx.od_pipeline(pcm)
    for i in (0, 4111, 8199):
        p1, a1, _ = ctx.od_pipeline(pcm[i:i + 1])
        assert np.array_equal(p1[0], p_all[i]) and a1[0] == a_all[i]
    base_si = synth.batch(1800, 24, 24000)
    pcm = np.tile(base_si, (342, 1))[:8200]
    p_all, a_all, _ = ctx.si_pipeline(pcm)
    for i in (1, 4100, 8198):
        p1, a1, _ = ctx.si_pipeline(pcm[i:i + 1])
        assert np.array_equal(p1[0], p_all[i]) and a1[0] == a_all[i]


@pytest.mark.parametrize('n', [1, 5, 32, 33, 200, 256])
def test_small_batch_lstm_split_bit_identical(monkeypatch, n):
    """Batches of <= 256 clips run the BiLSTM with each direction's hidden units spread over eight
    workgroups per 32 clips (nets.hip bilstm_h3_split_kernel, h exchanged through HBM each step); env
    MMLA_NO_LSTM_SPLIT=1 keeps one workgroup per direction.  Same bits, OD and SI, no NaN (a
    workgroup that gave up waiting writes NaN)."""
    from mmla_audio_amd import _lib, weights
    W = weights.synthetic(weights.OD, seed=23)
    Ws = weights.synthetic(weights.SI, seed=24, n_classes=630)
    od = synth.batch(1900 + n, n, 40000)
    si = [synth.clip(2000 + i, 24000 if i % 3 else 17000) for i in range(n)]
    out = []
    for flag in ('0', '1'):
        monkeypatch.setenv('MMLA_NO_LSTM_SPLIT', flag)
        monkeypatch.setenv('MMLA_LSTM_SPLIT_MAX', '256')   # the kernel's limit, past the default
        c = _lib.Context(0)
        monkeypatch.delenv('MMLA_NO_LSTM_SPLIT')
        monkeypatch.delenv('MMLA_LSTM_SPLIT_MAX')
        c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
        c.load_weights(weights.SI, weights.pack(weights.SI, Ws, 630), 630, _lib.HEAD_SOFTMAX)
        out.append((c.od_pipeline(od), c.si_pipeline(si)))
    (po, ao, _), (ps, as_, _) = out[0]
    (qo, bo, _), (qs, bs, _) = out[1]
    assert np.isfinite(po).all() and np.isfinite(ps).all()
    assert np.array_equal(po, qo) and np.array_equal(ao, bo)
    assert np.array_equal(ps, qs) and np.array_equal(as_, bs)


@pytest.mark.parametrize('n', [1, 3, 40])
def test_host_mapped_outputs_bit_identical(monkeypatch, n):
    """Small host-pointer calls gather their PCM (+ lens) into pinned memory for one DMA and write
    their outputs and the range flag into host-mapped memory (capi.cpp pin_small); env
    MMLA_NO_PIN_OUT=1 copies from pageable memory and stages outputs in HBM.  Same results for the
    pipelines, ragged (lens) input, overlapping windows, the front-end images and the network-only
    entry."""
    from mmla_audio_amd import _lib, weights
    W = weights.synthetic(weights.OD, seed=25)
    Ws = weights.synthetic(weights.SI, seed=26, n_classes=8)
    od = synth.batch(2100 + n, n, 40000)
    si = [synth.clip(2200 + i, 24000 if i % 2 else 3000) for i in range(n)]
    res = []
    for flag in ('0', '1'):
        monkeypatch.setenv('MMLA_NO_PIN_OUT', flag)
        c = _lib.Context(0)
        monkeypatch.delenv('MMLA_NO_PIN_OUT')
        c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
        c.load_weights(weights.SI, weights.pack(weights.SI, Ws, 8), 8, _lib.HEAD_SIGMOID)
        f = c.od_features(od)
        # overlapping windows of one signal (segmentation with step < window): the span path
        g = c.od_features_strided(synth.clip(2300, 80000), n, 1000, 40000, db=False, norm=False)
        res.append((c.od_pipeline(od), c.si_pipeline(si), f, c.od_forward(f['img']), g))
    (a_od, a_si, a_f, a_x, a_g), (b_od, b_si, b_f, b_x, b_g) = res
    for k in a_g:
        assert np.array_equal(a_g[k], b_g[k]), k
    for u, v in zip(a_od + a_si, b_od + b_si):
        assert np.array_equal(u, v)
    for k in a_f:   # a silent clip's normalize_matrix is 0/0 = NaN (the reference's too)
        assert np.array_equal(a_f[k], b_f[k], equal_nan=a_f[k].dtype.kind == 'f'), k
    assert np.array_equal(a_x, b_x)


@pytest.mark.parametrize('n', [1, 40])
def test_lstm_split_timeout_recovers(monkeypatch, n):
    """VERDICT r4 weak #4 / ADVICE r4: a split-BiLSTM workgroup that gives up waiting for the others
    writes NaN and sets a timeout flag; the host must not return those NaNs as a result.  Env
    MMLA_DEBUG_LSTM_SPIN=-1 makes every workgroup give up at its first wait without polling
    (deterministic; a positive bound of one poll only times out if a race is lost):
    host-pointer calls re-run the micro-batch on the one-workgroup-per-direction kernel (the same
    bits as MMLA_NO_LSTM_SPLIT=1, counted by debug_counters), and a device-pointer call reports the
    timeout from mmla_synchronize instead of returning NaN silently."""
    import torch
    from mmla_audio_amd import _lib, weights
    W = weights.synthetic(weights.OD, seed=27)
    Ws = weights.synthetic(weights.SI, seed=28, n_classes=8)
    od = synth.batch(2400 + n, n, 40000)
    si = [synth.clip(2500 + i, 24000) for i in range(n)]
    ctxs = {}
    for key, env in (('ref', {'MMLA_NO_LSTM_SPLIT': '1'}), ('spin1', {'MMLA_DEBUG_LSTM_SPIN': '-1'})):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        c = _lib.Context(0)
        for k in env:
            monkeypatch.delenv(k)
        c.load_weights(weights.OD, weights.pack(weights.OD, W), 2)
        c.load_weights(weights.SI, weights.pack(weights.SI, Ws, 8), 8, _lib.HEAD_SIGMOID)
        ctxs[key] = c
    ref, dbg = ctxs['ref'], ctxs['spin1']
    po, ao, _ = ref.od_pipeline(od)
    ps, as_, _ = ref.si_pipeline(si)
    qo, bo, _ = dbg.od_pipeline(od)
    qs, bs, _ = dbg.si_pipeline(si)
    assert np.isfinite(qo).all() and np.isfinite(qs).all()
    assert np.array_equal(po, qo) and np.array_equal(ao, bo)
    assert np.array_equal(ps, qs) and np.array_equal(as_, bs)
    f32_reruns, split_reruns = dbg.debug_counters()
    assert f32_reruns == 0 and split_reruns >= 1, (f32_reruns, split_reruns)
    # device pointers: the NaN launch is reported, not returned as success
    x = torch.from_numpy(od).cuda()
    probs = torch.empty((n, 2), dtype=torch.float32, device='cuda')
    dbg.set_stream(torch.cuda.current_stream().cuda_stream)
    dbg.od_pipeline_dev(x.data_ptr(), n, 40000, 40000, probs=probs.data_ptr())
    with pytest.raises(_lib.MmlaError) as e:
        dbg.synchronize()
    assert e.value.code == -2 and 'timed out' in str(e.value)
    assert torch.isnan(probs).any()
    dbg.synchronize()   # the flag is cleared by the report
