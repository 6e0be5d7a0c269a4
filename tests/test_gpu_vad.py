"""GPU: silence removal and the PCM_16 write, through the C ABI.

  collector + rewrite   bit-exact vs the reference's own vad_collector / save_wave_file run with a
                        stub is_speech (tests/golden/vad_golden.npz)
  webrtcvad decisions   bit-exact vs oracle/webrtc_vad.py (the restated fixed-point algorithm;
                        parity unpinned vs the absent library), one stream over several items, many
                        independent streams, and the state carried across calls
  PCM_16                identical to (short) lrintf(32767 * y) computed in float32 on the host
"""
import os

import numpy as np
import pytest

from oracle import synth, vad as ovad, webrtc_vad

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'vad_golden.npz')


@pytest.fixture(scope='module')
def ctx():
    from mmla_audio_amd import _lib
    return _lib.Context(0)


def _clip(seed, n=40960):
    """voiced synth with silent gaps (and one near-silent stretch) -- VAD on and off"""
    rng = np.random.default_rng(seed)
    x = synth.clip(seed * 5, n).astype(np.int32)            # class 0: voiced
    a, b = sorted(rng.integers(0, n, 2))
    x[a:b] = rng.integers(-3, 4, b - a)
    c = int(rng.integers(0, n // 2))
    x[c:c + 4800] = 0
    return x.astype(np.int16)


def test_collector_matches_reference(ctx):
    g = np.load(GOLDEN)
    names = list(g['names'])
    pcm = [g[f'pcm_{i}'] for i in range(len(names))]
    flags = [g[f'flags_{i}'] for i in range(len(names))]
    out = ctx.vad_collect(pcm, flags)
    for i, name in enumerate(names):
        assert np.array_equal(out[i], g[f'out_{i}']), name


def test_one_stream_several_items(ctx):
    items = [_clip(s) for s in (1, 2, 3)] + [np.zeros(40960, np.int16), _clip(4, 12000)]
    ref = webrtc_vad.Vad(3)
    want = [ovad.remove_silence(x, ref.is_speech) for x in items]
    ctx.vad_reset(1, 3)
    out, flags = ctx.vad_remove_silence(items, items_per_stream=len(items))
    for i, (o, f) in enumerate(want):
        assert np.array_equal(flags[i], f), f'item {i}: frame decisions'
        assert np.array_equal(out[i], o), f'item {i}: voiced PCM'
    assert any(len(o) < len(x) for (o, _), x in zip(want, items))    # something was removed
    assert any(len(o) > 0 for o, _ in want)                           # and something kept


def test_independent_streams(ctx):
    streams = [[_clip(10 + 2 * s), _clip(11 + 2 * s, 24000)] for s in range(6)]
    ctx.vad_reset(6, 3)
    out, flags = ctx.vad_remove_silence([x for st in streams for x in st], items_per_stream=2)
    for s, st in enumerate(streams):
        ref = webrtc_vad.Vad(3)
        for k, x in enumerate(st):
            o, f = ovad.remove_silence(x, ref.is_speech)
            assert np.array_equal(flags[2 * s + k], f) and np.array_equal(out[2 * s + k], o), (s, k)


def test_lens_longer_than_row_rejected_or_clamped(ctx):
    """an item length above the row width (the stride) must not read the next item or
    write past the output.  Host call: MMLA_E_INVALID.  Device-pointer call (lens not visible to the
    host): the kernels clamp to the row, so the output stays inside its rows and the guard words
    behind the last row are untouched."""
    import torch
    from mmla_audio_amd import _lib
    x = np.stack([_clip(40), _clip(41)])
    ctx.vad_reset(2, 3)
    with pytest.raises(_lib.MmlaError):
        ctx.vad_remove_silence(x, lens=np.array([x.shape[1], x.shape[1] + 480], np.int32))

    n, L = x.shape
    dev = torch.device('cuda:0')
    pcm = torch.from_numpy(x).to(dev)
    lens = torch.tensor([L, 3 * L], dtype=torch.int32, device=dev)
    guard = 4096
    out = torch.full((n * L + guard,), 12345, dtype=torch.int16, device=dev)
    olen = torch.zeros(n, dtype=torch.int32, device=dev)
    nf = (L - 1) // 480
    speech = torch.zeros((n, nf), dtype=torch.uint8, device=dev)
    ctx.vad_reset(2, 3)
    rc = ctx.lib.mmla_vad_remove_silence(ctx.h, pcm.data_ptr(), n, L, lens.data_ptr(), L, 1,
                                         out.data_ptr(), olen.data_ptr(), speech.data_ptr(), nf,
                                         _lib.MMLA_DEVICE_PTR)
    torch.cuda.synchronize()
    assert rc == 0
    assert bool((out[n * L:] == 12345).all()), 'write past the last row'
    assert int(olen.max()) <= L
    # the clamped item (its own stream, fresh detector) equals the item at its true length
    o, _ = ovad.remove_silence(x[1], webrtc_vad.Vad(3).is_speech)
    got = out[L:L + int(olen[1])].cpu().numpy()
    assert np.array_equal(got, o)


def test_state_persists_across_calls(ctx):
    a, b = _clip(30), _clip(31)
    ctx.vad_reset(1, 3)
    _, fa = ctx.vad_remove_silence([a])
    _, fb = ctx.vad_remove_silence([b])
    ctx.vad_reset(1, 3)
    _, fab = ctx.vad_remove_silence([a, b], items_per_stream=2)
    assert np.array_equal(fa[0], fab[0]) and np.array_equal(fb[0], fab[1])
    ctx.vad_reset(1, 0)                  # another mode: the quality detector flags at least as much
    _, f0 = ctx.vad_remove_silence([a, b], items_per_stream=2)
    assert f0[0].sum() + f0[1].sum() >= fab[0].sum() + fab[1].sum()


def test_dropin_names(ctx):
    from mmla_audio_amd import vad as mv
    x = _clip(40)
    v = mv.Vad(3)
    segs = list(mv.vad_collector(16000, 30, 300, v, mv.frame_generator(30, x.tobytes(), 16000)))
    got = np.frombuffer(b''.join(segs), '<i2')
    want, _ = ovad.remove_silence(x, webrtc_vad.Vad(3).is_speech)
    assert np.array_equal(got, want)
    assert v.is_speech(np.zeros(480, np.int16).tobytes(), 16000) in (True, False)


def test_pcm16_matches_libsndfile_rule(ctx):
    rng = np.random.default_rng(5)
    y = np.concatenate([rng.uniform(-1.2, 1.2, 100000),
                        (np.arange(-40, 41) + 0.5) / 32767.0,        # exact .5 ties: to even
                        [0.0, -0.0, 1.0, -1.0]]).astype(np.float32)
    got = ctx.pcm16(y)
    want = (np.rint(np.float32(32767.0) * y).astype(np.int64) & 0xFFFF).astype(np.uint16).view(np.int16)
    assert np.array_equal(got, want)


def test_save_wave_file_chain(tmp_path, ctx):
    """record_on_pc.py save_wave_file(noise_reduce=True, silence_remove=True): gate, PCM_16, VAD.

    The gate is checked against the oracle to its own tolerance (test_gpu_noisereduce.py: ~1e-7 of
    the peak, i.e. ~3e-3 LSB, so a sample sitting on a rounding tie may land one LSB apart); the
    PCM_16 rule and the VAD are then checked bit-exactly on the GPU gate's own float output."""
    import scipy.io.wavfile as wavfile
    from mmla_audio_amd import vad as mv
    from mmla_audio_amd import noisereduce as mnr
    from oracle import noisereduce as onr
    x = _clip(50)
    noise = (0.01 * np.random.default_rng(6).standard_normal(32000)).astype(np.float32)
    v = mv.Vad(3)
    path = str(tmp_path / 'c.wav')
    mv.save_wave_file(path, [x.tobytes()], noise_reduce=True, silence_remove=True, noise=noise, vad=v)
    sr, got = wavfile.read(path)
    xf = (x / 32768.0).astype(np.float32)
    y = mnr.reduce_noise(y=xf, sr=16000, y_noise=noise, stationary=True)
    y_ref = onr.reduce_noise(xf, 16000, noise)
    err = np.abs(y.astype(np.float64) - y_ref) / (np.abs(y_ref).max() + 1e-12)
    assert np.quantile(err, 0.999) <= 1e-5 and err.max() <= 2e-2
    q = (np.rint(np.float32(32767.0) * y.astype(np.float32)).astype(np.int64) & 0xFFFF).astype(np.uint16).view(np.int16)
    want, _ = ovad.remove_silence(q, webrtc_vad.Vad(3).is_speech)
    assert sr == 16000 and np.array_equal(got, want)


def test_si_post_analysing_flow(tmp_path, ctx):
    """speaker_identification_post_processing.post_analysing on one conversation, against the run
    of the reference's own function with a stub is_speech and a stub model (sipost_golden.npz)"""
    from datetime import datetime
    from mmla_audio_amd import speaker_identification_post_processing as sp
    g = np.load(os.path.join(os.path.dirname(GOLDEN), 'sipost_golden.npz'))
    whole, n_seg, seg_len = g['whole'], int(g['n_segments']), int(g['segment_len'])
    segments = [whole[seg_len * j:seg_len * (j + 1)] for j in range(n_seg)]
    nf = [(len(s) - 1) // 480 for s in segments]
    flags = np.split(g['flags'], np.cumsum(nf)[:-1])

    class StubModel:
        def predict(self, x):
            p = np.full((len(x), 3), 0.1)
            p[np.arange(len(x)), (np.arange(len(x)) + 1) % 3] = 0.8
            return p

    spk = sp.speaker_id_dict_from_corpus(list(g['corpus_listing']))
    labels, probs, silent = sp.post_analyse_conversation(whole, segments, StubModel(), spk, ctx=ctx,
                                                         speech=flags)
    log = str(tmp_path / 'conv0.txt')
    sp.write_log(log, labels, start_time=datetime(2026, 10, 16, 12, 0, 0))
    assert open(log).read() == str(g['log'])
    # the real detector on the same conversation runs and yields a subset of silent segments
    labels2, _, silent2 = sp.post_analyse_conversation(whole, segments, StubModel(), spk, ctx=ctx)
    assert len(labels2) == len(labels) and all(0 <= i < n_seg for i in silent2)


def test_si_post_detector_state_carries_across_conversations(ctx):
    """the reference's module-level Vad(3) (speaker_identification_post_processing.py:26)
    keeps its adaptive state from one conversation to the next; post_analyse_conversation keeps the
    context's detector after its first call.  Checked against ONE oracle detector run over both
    conversations' segments in order."""
    from mmla_audio_amd import speaker_identification_post_processing as sp

    class StubModel:
        def predict(self, x):
            return np.full((len(x), 2), 0.5)

    convs = [[_clip(76 + 2 * c + k, 40960) for k in range(2)] for c in range(2)]
    ref = webrtc_vad.Vad(3)
    want = [[i for i, s in enumerate(segs) if len(ovad.remove_silence(s, ref.is_speech)[0]) < 4000]
            for segs in convs]
    got = []
    for c, segs in enumerate(convs):
        _, _, silent = sp.post_analyse_conversation(np.concatenate(segs), segs, StubModel(),
                                                    {'0': 'a', '1': 'b'}, ctx=ctx, reset_vad=(c == 0))
        got.append(list(silent))
    assert got == want
    # the carried state matters on this input: a fresh detector on the second conversation decides
    # at least one frame differently than the one that saw the first conversation
    ref_c = webrtc_vad.Vad(3)
    for s_ in convs[0]:
        ovad.remove_silence(s_, ref_c.is_speech)
    carried = [ovad.remove_silence(s_, ref_c.is_speech)[1] for s_ in convs[1]]
    fresh = webrtc_vad.Vad(3)
    alone = [ovad.remove_silence(s_, fresh.is_speech)[1] for s_ in convs[1]]
    assert any(not np.array_equal(a, b) for a, b in zip(carried, alone))
