"""GPU parity tests: the HIP path (through the C ABI) against the reference fixtures and the
oracle. Tolerances (fp32): mel / frames <= 1e-4 L-inf (north_star), waveforms <= 1e-4 L-inf,
stop steps and alignment argmax bit-exact (argmax only where the reference's top-2 margin
exceeds 1e-5; ties below that are implementation-defined in fp32).
"""
import os

import numpy as np
import pytest
import torch

from helpers import (build_melgan, build_taco, load_fixture, melgan_oracle, melgan_state_dict,
                     taco_state_dict)
from tts_amd.spec import tacotron2_spec
from tts_amd.weights import synth_state_dict

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MEL_TOL = 1e-4
WAV_TOL = 1e-4
ALIGN_MARGIN = 1e-5


def _dev():
    if not torch.cuda.is_available():
        pytest.fail("GPU test requires a ROCm device")
    return torch.device("cuda:0")


# ------------------------------------------------------------------------------- PQMF
def test_pqmf_synthesis_matches_reference():
    from tts_amd import PQMF
    dev = _dev()
    fx = load_fixture("pqmf")
    p = PQMF().to(dev)
    assert np.array_equal(p.G.cpu().numpy(), fx["G"])
    y = p.synthesis(torch.from_numpy(fx["x"]).to(dev)).cpu().numpy()
    assert y.shape == fx["y"].shape
    assert np.abs(y - fx["y"]).max() <= 1e-5


def test_pqmf_known_answer_wav():
    """TTS/vocoder/pqmf_output.wav (reference's committed output) within int16 rounding."""
    from tts_amd import PQMF
    dev = _dev()
    fx = load_fixture("pqmf")
    y = PQMF().to(dev).synthesis(torch.from_numpy(fx["example_bands"]).to(dev)).cpu().numpy()[0, 0]
    assert np.abs(y - fx["example_rec"][0, 0]).max() <= 1e-5
    ka = fx["known_answer_int16"].astype(np.float64)
    n = len(ka) - 64
    pcm = y[:n].astype(np.float64) * 32768.0
    assert np.abs(pcm - ka[:n]).max() <= 2.0


# ------------------------------------------------------------------------------ MelGAN
@pytest.fixture(scope="module")
def melgan():
    dev = _dev()
    fx = load_fixture("mbmelgan")
    cfg, sd = melgan_state_dict(int(fx["seed"]))
    return fx, cfg, sd, build_melgan(cfg, sd, dev)


@pytest.mark.parametrize("key", ["M7_p0", "M64_p0", "M5_p2", "M33_p2"])
def test_mbmelgan_inference_matches_reference(melgan, key):
    fx, cfg, sd, v = melgan
    v.inference_padding = int(key.split("_p")[1])
    mel = torch.from_numpy(fx[key + "_mel"]).cuda()
    wav = v.inference(mel).cpu().numpy()
    ref = fx[key + "_wav"]
    assert wav.shape == ref.shape
    assert np.abs(wav - ref).max() <= WAV_TOL
    bands = v.generator(mel).cpu().numpy()
    assert np.abs(bands - fx[key + "_bands"]).max() <= WAV_TOL


def test_mbmelgan_batched_equals_single(melgan):
    fx, cfg, sd, v = melgan
    v.inference_padding = 0
    mels = [fx["M64_p0_mel"][0], fx["M7_p0_mel"][0]]
    M = max(m.shape[1] for m in mels)
    batch = np.zeros((2, 80, M), np.float32)
    for i, m in enumerate(mels):
        batch[i, :, :m.shape[1]] = m
    wav = v.inference(torch.from_numpy(batch).cuda(), lengths=[64, 7]).cpu().numpy()
    for i, key in enumerate(["M64_p0", "M7_p0"]):
        ref = fx[key + "_wav"][0, 0]
        assert np.abs(wav[i, 0, :len(ref)] - ref).max() <= WAV_TOL
        assert not wav[i, 0, len(ref):].any()


def test_mbmelgan_writes_zero_padding_itself(melgan):
    """The fused output stage (melgan_out.hip out_pqmf_kernel) writes every row's samples up to the
    padded length, zeros past the row's own length (whole tiles past it included), so the caller's
    buffer needs no memset: a NaN-filled buffer comes back with the same samples as the batched
    call and exact zeros in the padding."""
    from tts_amd._lib import get_engine
    fx, cfg, sd, v = melgan
    v.inference_padding = 0
    mels = [fx["M64_p0_mel"][0], fx["M7_p0_mel"][0]]
    batch = np.zeros((2, 80, 64), np.float32)
    for i, m in enumerate(mels):
        batch[i, :, :m.shape[1]] = m
    x = torch.from_numpy(batch).cuda()
    ref = v.inference(x, lengths=[64, 7])
    wav = torch.full_like(ref, float("nan"))
    eng = get_engine(x.device)
    with eng.lock:
        v._sync(eng)
        eng.melgan_infer(x, np.array([64, 7]), 0, wav)
    torch.cuda.synchronize()
    assert not torch.isnan(wav).any()
    assert torch.equal(wav, ref)
    assert not wav[1, 0, v.hop * 7:].any()  # 3 whole 1008-position tiles past row 1's 448


def test_mbmelgan_random_vs_oracle(melgan):
    fx, cfg, sd, v = melgan
    orc = melgan_oracle(cfg, sd)
    rs = np.random.RandomState(3)
    lens = [9, 23, 4]
    M = max(lens)
    batch = np.zeros((3, 80, M), np.float32)
    for i, L in enumerate(lens):
        batch[i, :, :L] = rs.normal(0, 1.5, (80, L))
    v.inference_padding = 1
    wav = v.inference(torch.from_numpy(batch).cuda(), lengths=lens).cpu().numpy()
    for i, L in enumerate(lens):
        ref = orc.inference(batch[i, :, :L], pad=1)[0]
        assert np.abs(wav[i, 0, :len(ref)] - ref).max() <= WAV_TOL


def _gemm(mode):
    from tts_amd._lib import get_engine
    eng = get_engine(torch.device("cuda:0"))
    eng.set_gemm_mode(mode)
    return eng


def test_mbmelgan_split_f16_equals_fp32_path_and_oracle(melgan):
    """The split-f16 ResidualStack kernels (default) against the fp32-MFMA kernels and the oracle
    on ragged utterances long enough for every dilation: both paths within WAV_TOL of the oracle,
    and the split path's error no more than twice the fp32 path's (the same error class)."""
    fx, cfg, sd, v = melgan
    orc = melgan_oracle(cfg, sd)
    rs = np.random.RandomState(8)
    lens = [61, 7, 40]
    batch = np.zeros((3, 80, max(lens)), np.float32)
    for i, L in enumerate(lens):
        batch[i, :, :L] = rs.normal(0, 1.5, (80, L))
    v.inference_padding = 0
    x = torch.from_numpy(batch).cuda()
    eng = _gemm("f32")
    try:
        w32 = v.inference(x, lengths=lens).cpu().numpy()
    finally:
        eng = _gemm("x3")
    n0 = eng.gemm_mode()[1]
    w16 = v.inference(x, lengths=lens).cpu().numpy()
    assert eng.gemm_mode() == ("x3", n0)  # no range fallback on this input
    e16 = e32 = 0.0
    for i, L in enumerate(lens):
        ref = orc.inference(batch[i, :, :L], pad=0)[0]
        e16 = max(e16, float(np.abs(w16[i, 0, :len(ref)] - ref).max()))
        e32 = max(e32, float(np.abs(w32[i, 0, :len(ref)] - ref).max()))
        assert not w16[i, 0, len(ref):].any()
    print(f"waveform error vs oracle: split-f16 {e16:.2e}, fp32 {e32:.2e}, between {np.abs(w16 - w32).max():.2e}")
    assert e16 <= WAV_TOL and e32 <= WAV_TOL
    assert e16 <= 2 * e32 + 2e-6  # same error class as the fp32 GEMM


def test_mbmelgan_f16_range_fallback_reruns_in_fp32(melgan):
    """An input that drives the ResidualStack operands past the f16 range (|v| >= 65504) raises the
    range flag and the call is re-run on the fp32 kernels: the result is bit-identical to the
    fp32-mode call and the fallback counter moves."""
    fx, cfg, sd, v = melgan
    v.inference_padding = 0
    mel = torch.from_numpy(fx["M64_p0_mel"] * np.float32(1e5)).cuda()
    eng = _gemm("f32")
    try:
        w32 = v.inference(mel).cpu().numpy()
    finally:
        eng = _gemm("x3")
    n0 = eng.gemm_mode()[1]
    w16 = v.inference(mel).cpu().numpy()
    assert eng.gemm_mode()[1] == n0 + 1
    assert np.array_equal(w16, w32)


@pytest.mark.parametrize("mode", ["x3", "f32"])
def test_mbmelgan_frame_major_view_equals_contiguous(melgan, mode):
    """A (B, M, 80) postnet-style tensor passed as its (B, 80, M) transposed view is read in place
    (tts_melgan_infer_strided, no copy): bit-identical to the contiguous call on both GEMM paths,
    replicate padding included, and within WAV_TOL of the oracle."""
    fx, cfg, sd, v = melgan
    orc = melgan_oracle(cfg, sd)
    rs = np.random.RandomState(11)
    lens = [37, 6, 21]
    fm = np.zeros((3, max(lens), 80), np.float32)  # frame-major
    for i, L in enumerate(lens):
        fm[i, :L] = rs.normal(0, 1.5, (L, 80))
    view = torch.from_numpy(fm).cuda().transpose(1, 2)
    assert not view.is_contiguous()
    eng = _gemm(mode)
    try:
        for pad in (0, 2):
            v.inference_padding = pad
            w_view = v.inference(view, lengths=lens).cpu().numpy()
            w_cont = v.inference(view.contiguous(), lengths=lens).cpu().numpy()
            assert np.array_equal(w_view, w_cont)
            for i, L in enumerate(lens):
                ref = orc.inference(np.ascontiguousarray(fm[i, :L].T), pad=pad)[0]
                assert np.abs(w_view[i, 0, :len(ref)] - ref).max() <= WAV_TOL
    finally:
        _gemm("x3")
        v.inference_padding = 0


@pytest.mark.parametrize("mode", ["x3", "f32"])
def test_fullband_melgan_generator_vs_oracle(mode):
    """MelganGenerator as setup_generator builds the reference's "melgan_generator" (base 512,
    upsampling 8x8x2x2, 3 residual blocks: ResidualStacks at C = 256 / 128 / 64 / 32, the split-f16
    block kernel's R = 4 / 4 / 2 / 1 weight rings) against the numpy oracle on a ragged batch, on
    both GEMM paths; samples past each utterance's length are zero."""
    from tts_amd import MelganGenerator
    from tts_amd.spec import MelganConfig
    _dev()
    cfg, sd = melgan_state_dict(7, MelganConfig(out_channels=1, base_channels=512, upsample_factors=(8, 8, 2, 2),
                                                num_res_blocks=3, pqmf=False))
    v = MelganGenerator(in_channels=80, out_channels=1, base_channels=512, upsample_factors=(8, 8, 2, 2),
                        num_res_blocks=3)
    full = v.state_dict()
    full.update({k: torch.from_numpy(t) for k, t in sd.items()})
    v.load_state_dict(full)
    v.remove_weight_norm()
    v = v.cuda().eval()
    v.inference_padding = 0
    orc = melgan_oracle(cfg, sd)
    rs = np.random.RandomState(4)
    lens = [13, 5, 9]
    batch = np.zeros((3, 80, max(lens)), np.float32)
    for i, L in enumerate(lens):
        batch[i, :, :L] = rs.normal(0, 1.5, (80, L))
    eng = _gemm(mode)
    try:
        n0 = eng.gemm_mode()[1]
        wav = v.inference(torch.from_numpy(batch).cuda(), lengths=lens).cpu().numpy()
        assert eng.gemm_mode() == (mode, n0)  # no range fallback on this input
    finally:
        _gemm("x3")
    for i, L in enumerate(lens):
        ref = orc.generator(batch[i, :, :L])
        assert wav[i, 0, :ref.shape[1]].shape == ref[0].shape
        assert np.abs(wav[i, 0, :ref.shape[1]] - ref[0]).max() <= WAV_TOL
        assert not wav[i, 0, ref.shape[1]:].any()


def test_fullband_default_odd_length_unaligned_rows_vs_oracle():
    """FullbandMelganGenerator's own defaults (base 512, upsampling 2x8x2x2, 4 residual blocks,
    inference padding 2): an odd mel length makes the first stage's row length 2 (M + 4) not a
    multiple of 4, so the split-f16 block kernel stores per position instead of 16 bytes at a time
    (this shape used to raise). Against the oracle, ragged, padding 2."""
    from tts_amd import FullbandMelganGenerator
    from tts_amd.spec import MelganConfig
    _dev()
    cfg, sd = melgan_state_dict(9, MelganConfig(out_channels=1, base_channels=512, upsample_factors=(2, 8, 2, 2),
                                                num_res_blocks=4, pqmf=False))
    v = FullbandMelganGenerator()
    full = v.state_dict()
    full.update({k: torch.from_numpy(t) for k, t in sd.items()})
    v.load_state_dict(full)
    v.remove_weight_norm()
    v = v.cuda().eval()
    assert v.inference_padding == 2
    orc = melgan_oracle(cfg, sd)
    rs = np.random.RandomState(5)
    lens = [13, 11]  # odd: stage 0 rows of 2 (13 + 4) = 34 floats; > the dilation-27 reflection pad
    batch = np.zeros((2, 80, max(lens)), np.float32)
    for i, L in enumerate(lens):
        batch[i, :, :L] = rs.normal(0, 1.5, (80, L))
    with pytest.raises(RuntimeError, match="ReflectionPad1d"):  # 2 (9 + 4) = 26 <= 27, as torch raises
        v.inference(torch.from_numpy(batch[:1, :, :9]).cuda())
    wav = v.inference(torch.from_numpy(batch).cuda(), lengths=lens).cpu().numpy()
    for i, L in enumerate(lens):
        c = batch[i, :, :L]
        c = np.concatenate([np.repeat(c[:, :1], 2, 1), c, np.repeat(c[:, -1:], 2, 1)], 1)  # replicate pad
        ref = orc.generator(c).reshape(-1)
        assert ref.size == 64 * (L + 4)  # hop 2 x 8 x 2 x 2
        assert np.abs(wav[i, 0, :ref.size] - ref).max() <= WAV_TOL, i
        assert not wav[i, 0, ref.size:].any()


def test_mbmelgan_too_short_raises(melgan):
    fx, cfg, sd, v = melgan
    v.inference_padding = 0
    with pytest.raises(RuntimeError):
        v.inference(torch.zeros(1, 80, 3, device="cuda"))


# --------------------------------------------------------------------------- Tacotron2
@pytest.fixture(scope="module")
def taco_sig():
    _dev()
    return load_fixture("taco_sigmoid")


def test_encoder_matches_reference(taco_sig):
    from tts_amd._lib import get_engine
    fx = taco_sig
    cfg, sd = taco_state_dict(fx, r=2)
    m = build_taco(cfg, sd)
    eng = get_engine("cuda:0")
    m._sync(eng)
    ids = [fx["r2_u0_ids"], fx["r2_u1_ids"], fx["r2_u2_ids"]]
    T = max(len(x) for x in ids)
    batch = np.zeros((3, T), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    out = torch.empty(3, T, 512, device="cuda")
    eng.taco_encoder(torch.from_numpy(batch).cuda(), [len(x) for x in ids], out)
    enc = out[1, :len(ids[1])].cpu().numpy()
    assert np.abs(enc - fx["r2_u1_enc"]).max() <= 1e-5
    assert not out[1, len(ids[1]):].any()


@pytest.mark.parametrize("B", [32, 64, 24])
def test_encoder_row_groups_vs_oracle(B):
    """The persistent BiLSTM's row groups (B = 17..32 and 49..64 run as two independent recurrences
    per direction on all 256 CUs): every row's encoder output against the oracle encoder at B = 1,
    ragged lengths up to the LJ maximum, zero past each length."""
    from oracle.taco_np import TacoOracle
    from tts_amd._lib import get_engine
    from tts_amd.spec import TacotronConfig
    _dev()
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=4, overrides={}, stop_bias=-1e4, cfg=cfg)
    m = build_taco(cfg, sd)
    eng = get_engine("cuda:0")
    m._sync(eng)
    rs = np.random.RandomState(B)
    lens = rs.randint(2, 169, size=B)
    lens[B // 3] = 168
    ids = [rs.randint(1, 129, size=L).astype(np.int64) for L in lens]
    T = int(lens.max())
    batch = np.zeros((B, T), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    out = torch.empty(B, T, 512, device="cuda")
    eng.taco_encoder(torch.from_numpy(batch).cuda(), [int(L) for L in lens], out)
    out = out.cpu().numpy()
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    for i in range(B):
        ref = orc.encoder(ids[i])
        assert np.abs(out[i, :lens[i]] - ref).max() <= 1e-5, i
        assert not out[i, lens[i]:].any(), i


@pytest.mark.gpu
def test_bilstm_row_group_barrier_timeout_raises(monkeypatch):
    """A grid-barrier timeout in the BiLSTM's second row group (recurrence 3: row group 1, backward;
    B = 32 runs 2 row groups x 2 directions) is reported by the Tacotron2 call's status read-back:
    the call raises instead of returning mels built from a half-written encoder output.
    The test hook tts_test_stall_lstm (a C-ABI call, no environment variable) makes one workgroup of that recurrence leave before its second
    barrier. The next call, without the hook, is correct again."""
    from oracle.taco_np import TacoOracle
    from tts_amd.spec import TacotronConfig
    _dev()
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=4, overrides={}, stop_bias=-1e4, cfg=cfg)
    m = build_taco(cfg, sd)
    m.decoder.set_r(2)
    rs = np.random.RandomState(7)
    lens = rs.randint(8, 40, size=32)
    batch = np.zeros((32, int(lens.max())), np.int64)
    for i, L in enumerate(lens):
        batch[i, :L] = rs.randint(1, 129, size=L)
    x = torch.from_numpy(batch).cuda()
    from tts_amd._lib import load_library
    lib = load_library()
    lib.tts_test_stall_lstm(3)
    try:
        with pytest.raises(RuntimeError, match="persistent BiLSTM: grid barrier timed out"):
            m.inference(x, text_lengths=[int(L) for L in lens], max_decoder_steps=3)
    finally:
        lib.tts_test_stall_lstm(-1)
    dec, post, align, stop = m.inference(x, text_lengths=[int(L) for L in lens], max_decoder_steps=3)
    post = post.cpu().numpy()
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    for i in (0, 31):
        _, p, _, _ = orc.inference(batch[i, :lens[i]], 2, 3)
        assert np.abs(post[i, :len(p)] - p).max() <= MEL_TOL


def _check_taco(fx, r, dec, post, align, stop, steps, utts):
    for i in utts:
        k = f"r{r}_u{i}"
        S = len(fx[k + "_stop"])
        assert steps[i] == S, f"{k}: steps {steps[i]} != reference {S}"
        M = S * r
        assert np.abs(dec[i, :M] - fx[k + "_dec"]).max() <= MEL_TOL
        assert np.abs(post[i, :M] - fx[k + "_post"]).max() <= MEL_TOL
        assert not post[i, M:].any() and not dec[i, M:].any()
        a = align[i, :S, :fx[k + "_align"].shape[1]]
        assert np.abs(a - fx[k + "_align"]).max() <= 1e-5
        sel = fx[k + "_top2"] > ALIGN_MARGIN
        assert np.array_equal(a.argmax(1)[sel], fx[k + "_align"].argmax(1)[sel])
        assert np.abs(stop[i, :S, 0] - fx[k + "_stop"]).max() <= 1e-4


@pytest.mark.parametrize("r", [2, 1])
def test_tacotron2_batched_matches_reference(taco_sig, r):
    fx = taco_sig
    cfg, sd = taco_state_dict(fx, r=r)
    m = build_taco(cfg, sd)
    m.decoder.set_r(r)
    m.decoder.max_decoder_steps = int(fx[f"r{r}_max_steps"])
    ids = [fx[f"r{r}_u{i}_ids"] for i in range(3)]
    T = max(len(x) for x in ids)
    batch = np.zeros((3, T), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    dec, post, align, stop = m.inference(torch.from_numpy(batch).cuda(), text_lengths=[len(x) for x in ids])
    _check_taco(fx, r, dec.cpu().numpy(), post.cpu().numpy(), align.cpu().numpy(), stop.cpu().numpy(),
                m.last_steps, range(3))


def test_tacotron2_bidirectional_decoder_checkpoint(taco_sig):
    """bidirectional_decoder=True adds decoder_backward.* (a deepcopy of the decoder,
    tacotron_abstract.py:104-105) that inference never runs: same frames as the reference."""
    import dataclasses
    fx = taco_sig
    cfg, sd = taco_state_dict(fx, r=2)
    cfg = dataclasses.replace(cfg, bidirectional_decoder=True)
    full = synth_state_dict(tacotron2_spec(cfg), 99)
    full.update(sd)  # the fixture's weights; decoder_backward.* stay random
    m = build_taco(cfg, full)
    m.decoder.set_r(2)
    m.decoder.max_decoder_steps = int(fx["r2_max_steps"])
    ids = [fx[f"r2_u{i}_ids"] for i in range(3)]
    T = max(len(x) for x in ids)
    batch = np.zeros((3, T), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    dec, post, align, stop = m.inference(torch.from_numpy(batch).cuda(), text_lengths=[len(x) for x in ids])
    _check_taco(fx, 2, dec.cpu().numpy(), post.cpu().numpy(), align.cpu().numpy(), stop.cpu().numpy(),
                m.last_steps, range(3))


@pytest.mark.parametrize("name,n", [("taco_multispk", 3), ("taco_extspk", 2), ("taco_graves_spk", 2)])
def test_tacotron2_multispeaker_matches_reference(name, n):
    """Multi-speaker Tacotron2 (models/tacotron2.py:50-58,152-155), every utterance of the fixture
    in ONE batched call with its own speaker: learned table ids, or external 256-d embeddings."""
    _dev()
    fx = load_fixture(name)
    r = 2
    cfg, sd = taco_state_dict(fx, r=r)
    m = build_taco(cfg, sd)
    m.decoder.set_r(r)
    m.decoder.max_decoder_steps = int(fx[f"r{r}_max_steps"])
    ids = [fx[f"r{r}_u{i}_ids"] for i in range(n)]
    spk = [fx[f"r{r}_u{i}_spk"] for i in range(n)]
    T = max(len(x) for x in ids)
    batch = np.zeros((n, T), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    kw = ({"speaker_embeddings": torch.from_numpy(np.stack(spk)).cuda()} if spk[0].ndim
          else {"speaker_ids": torch.tensor([int(x) for x in spk])})
    dec, post, align, stop = m.inference(torch.from_numpy(batch).cuda(), text_lengths=[len(x) for x in ids], **kw)
    _check_taco(fx, r, dec.cpu().numpy(), post.cpu().numpy(), align.cpu().numpy(), stop.cpu().numpy(),
                m.last_steps, range(n))


@pytest.mark.parametrize("name", ["taco_bnprenet", "taco_window", "taco_window_softmax", "taco_fwdattn",
                                  "taco_fwdmask", "taco_graves"])
def test_tacotron2_decoder_variants_match_reference(name):
    """SURVEY 8f rank 4 decoder variants on the persistent decoder, both fixture utterances in one
    batched call: BN prenet, attention windowing (sigmoid / softmax), forward attention with the
    transition agent."""
    _dev()
    fx = load_fixture(name)
    r = 2
    cfg, sd = taco_state_dict(fx, r=r)
    m = build_taco(cfg, sd)
    m.decoder.set_r(r)
    m.decoder.max_decoder_steps = int(fx[f"r{r}_max_steps"])
    ids = [fx[f"r{r}_u{i}_ids"] for i in range(2)]
    T = max(len(x) for x in ids)
    batch = np.zeros((2, T), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    dec, post, align, stop = m.inference(torch.from_numpy(batch).cuda(), text_lengths=[len(x) for x in ids])
    _check_taco(fx, r, dec.cpu().numpy(), post.cpu().numpy(), align.cpu().numpy(), stop.cpu().numpy(),
                m.last_steps, range(2))


def test_tacotron2_multispeaker_requires_speaker():
    _dev()
    fx = load_fixture("taco_multispk")
    cfg, sd = taco_state_dict(fx, r=2)
    m = build_taco(cfg, sd)
    ids = torch.from_numpy(fx["r2_u0_ids"][None]).cuda()
    with pytest.raises(ValueError):
        m.inference(ids)
    with pytest.raises(IndexError):
        m.inference(ids, speaker_ids=torch.tensor([4]))


@pytest.mark.parametrize("u", [0, 1, 2])
def test_tacotron2_single_utterance_matches_reference(taco_sig, u):
    fx = taco_sig
    r = 2
    cfg, sd = taco_state_dict(fx, r=r)
    m = build_taco(cfg, sd)
    m.decoder.set_r(r)
    m.decoder.max_decoder_steps = int(fx[f"r{r}_max_steps"])
    ids = fx[f"r{r}_u{u}_ids"]
    dec, post, align, stop = m.inference(torch.from_numpy(ids[None]).cuda())
    S = len(fx[f"r{r}_u{u}_stop"])
    assert dec.shape == (1, S * r, 80) and align.shape == (1, S, len(ids)) and stop.shape == (1, S, 1)
    k = f"r{r}_u{u}"
    assert np.abs(dec[0].cpu().numpy() - fx[k + "_dec"]).max() <= MEL_TOL
    assert np.abs(post[0].cpu().numpy() - fx[k + "_post"]).max() <= MEL_TOL


def test_tacotron2_softmax_matches_reference():
    _dev()
    fx = load_fixture("taco_softmax")
    r = 2
    cfg, sd = taco_state_dict(fx, r=r)
    m = build_taco(cfg, sd)
    m.decoder.set_r(r)
    m.decoder.max_decoder_steps = int(fx[f"r{r}_max_steps"])
    ids = [fx[f"r{r}_u{i}_ids"] for i in range(2)]
    T = max(len(x) for x in ids)
    batch = np.zeros((2, T), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    dec, post, align, stop = m.inference(torch.from_numpy(batch).cuda(), text_lengths=[len(x) for x in ids])
    _check_taco(fx, r, dec.cpu().numpy(), post.cpu().numpy(), align.cpu().numpy(), stop.cpu().numpy(),
                m.last_steps, range(2))


def test_tacotron2_random_batch_vs_oracle():
    """Seeded xavier-scale model, 6 ragged utterances, forced length (stop bias -1e4)."""
    from oracle.taco_np import TacoOracle
    from tts_amd.spec import TacotronConfig
    _dev()
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=11, overrides={}, stop_bias=-1e4, cfg=cfg)
    m = build_taco(cfg, sd)
    r = 2
    m.decoder.set_r(r)
    rs = np.random.RandomState(4)
    lens = [17, 5, 40, 1, 29, 12]
    steps = [9, 14, 6, 3, 11, 7]
    T = max(lens)
    batch = np.zeros((len(lens), T), np.int64)
    for i, L in enumerate(lens):
        batch[i, :L] = rs.randint(1, 129, L)
    dec, post, align, stop = m.inference(torch.from_numpy(batch).cuda(), text_lengths=lens, max_decoder_steps=steps)
    assert list(m.last_steps) == steps
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    dec, post, align = dec.cpu().numpy(), post.cpu().numpy(), align.cpu().numpy()
    for i, L in enumerate(lens):
        d, p, a, s = orc.inference(batch[i, :L], r, steps[i])
        M = steps[i] * r
        assert np.abs(dec[i, :M] - d).max() <= MEL_TOL
        assert np.abs(post[i, :M] - p).max() <= MEL_TOL
        assert np.abs(align[i, :steps[i], :L] - a).max() <= 1e-5
        assert not align[i, :, L:].any()


def _taco_random_batch(seed, scale_embedding=1.0):
    from tts_amd.spec import TacotronConfig
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=seed, overrides={}, stop_bias=-1e4, cfg=cfg)
    if scale_embedding != 1.0:
        sd["embedding.weight"] = sd["embedding.weight"] * scale_embedding
    m = build_taco(cfg, sd)
    m.decoder.set_r(2)
    rs = np.random.RandomState(5)
    lens = [23, 4, 37, 11]
    steps = [8, 5, 12, 6]
    batch = np.zeros((len(lens), max(lens)), np.int64)
    for i, L in enumerate(lens):
        batch[i, :L] = rs.randint(1, 129, L)
    return cfg, sd, m, batch, lens, steps


def test_tacotron2_split_f16_equals_fp32_path_and_oracle():
    """Encoder convs, BiLSTM input projection, processed inputs and postnet on the split-f16 conv
    kernel (conv_x3.hip, the default) against the fp32-MFMA kernels and the oracle: both within
    MEL_TOL, the split path's error no more than twice the fp32 path's plus 2e-6 (the same error
    class), stop steps identical, no range fallback."""
    from oracle.taco_np import TacoOracle
    _dev()
    cfg, sd, m, batch, lens, steps = _taco_random_batch(13)
    x = torch.from_numpy(batch).cuda()
    eng = _gemm("f32")
    try:
        _, p32, a32, _ = m.inference(x, text_lengths=lens, max_decoder_steps=steps)
    finally:
        eng = _gemm("x3")
    n0 = eng.gemm_mode()[1]
    _, p16, a16, _ = m.inference(x, text_lengths=lens, max_decoder_steps=steps)
    assert eng.gemm_mode() == ("x3", n0)
    assert list(m.last_steps) == steps
    p32, p16, a16 = p32.cpu().numpy(), p16.cpu().numpy(), a16.cpu().numpy()
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    e16 = e32 = 0.0
    for i, L in enumerate(lens):
        _, p, a, _ = orc.inference(batch[i, :L], 2, steps[i])
        M = steps[i] * 2
        e16 = max(e16, float(np.abs(p16[i, :M] - p).max()))
        e32 = max(e32, float(np.abs(p32[i, :M] - p).max()))
        assert (a16[i, :steps[i], :L].argmax(1) == a.argmax(1)).all()
        assert not p16[i, M:].any()
    print(f"postnet error vs oracle: split-f16 {e16:.2e}, fp32 {e32:.2e}")
    assert e16 <= MEL_TOL and e32 <= MEL_TOL
    assert e16 <= 2 * e32 + 2e-6


@pytest.mark.parametrize("r", [2, 1])
def test_tacotron2_amplified_regime_split_f16_vs_fp32(r):
    """SURVEY 7's mildly amplified decoder regime (fixture taco_amplified: LSTM weights x2.1,
    projection x10, attention v x6; the reference's own fp32-vs-fp64 drift reaches 3-5e-6 at r=2 and
    1-3e-5 at r=1), where a reduced-precision decoder GEMM would show first. Both GEMM modes, the
    whole fixture in one batched call: mel <= 1e-4 against the reference, stop steps exact, argmax
    exact above the margin, and the split-f16 path's error against the reference's fp64 run no more
    than twice the fp32-MFMA path's plus 2e-6 (models/layers/tacotron2.py:259-298)."""
    _dev()
    fx = load_fixture("taco_amplified")
    cfg, sd = taco_state_dict(fx, r=r)
    m = build_taco(cfg, sd)
    m.decoder.set_r(r)
    m.decoder.max_decoder_steps = int(fx[f"r{r}_max_steps"])
    ids = [fx[f"r{r}_u{i}_ids"] for i in range(3)]
    batch = np.zeros((3, max(len(x) for x in ids)), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    x = torch.from_numpy(batch).cuda()
    err64 = {}
    for mode in ("f32", "x3"):
        eng = _gemm(mode)
        try:
            n0 = eng.gemm_mode()[1]
            dec, post, align, stop = m.inference(x, text_lengths=[len(t) for t in ids])
            assert eng.gemm_mode() == (mode, n0)  # no range fallback
        finally:
            _gemm("x3")
        post = post.cpu().numpy()
        _check_taco(fx, r, dec.cpu().numpy(), post, align.cpu().numpy(), stop.cpu().numpy(), m.last_steps, range(3))
        err64[mode] = max(float(np.abs(post[i, :len(fx[f"r{r}_u{i}_post64"])] - fx[f"r{r}_u{i}_post64"]).max())
                          for i in range(3))
    drift = max(float(fx[f"r{r}_u{i}_drift64"]) for i in range(3))
    print(f"r={r} error vs fp64: split-f16 {err64['x3']:.2e}, fp32 {err64['f32']:.2e}, reference fp32 {drift:.2e}")
    assert err64["x3"] <= 2 * err64["f32"] + 2e-6


def test_tacotron2_f16_range_fallback_reruns_in_fp32():
    """An embedding table scaled far past the f16 range drives the encoder conv operands over 65504:
    the split-f16 call raises its range flag and re-runs on the fp32 kernels, bit-identical to the
    fp32-mode call, and the fallback counter moves."""
    _dev()
    cfg, sd, m, batch, lens, steps = _taco_random_batch(13, scale_embedding=1e8)
    x = torch.from_numpy(batch).cuda()
    eng = _gemm("f32")
    try:
        out32 = [t.cpu().numpy() for t in m.inference(x, text_lengths=lens, max_decoder_steps=steps)]
    finally:
        eng = _gemm("x3")
    n0 = eng.gemm_mode()[1]
    out16 = [t.cpu().numpy() for t in m.inference(x, text_lengths=lens, max_decoder_steps=steps)]
    assert eng.gemm_mode()[1] == n0 + 1
    for u, v in zip(out16, out32):
        assert np.array_equal(u, v, equal_nan=True)


@pytest.mark.parametrize("variant", ["graves", "fwdmask", "window_softmax"])
def test_tacotron2_variant_random_batch_vs_oracle(variant):
    """Decoder variants on 6 ragged utterances (1 to 40 tokens, forced lengths) against the oracle:
    Graves attention, forward attention with the mask (its Python index wrap fires on short rows),
    softmax windowing."""
    from oracle.taco_np import TacoOracle
    from tts_amd.spec import TacotronConfig
    _dev()
    kw = {"graves": dict(attn_type="graves"),
          "fwdmask": dict(forward_attn=True, trans_agent=True, forward_attn_mask=True),
          "window_softmax": dict(attn_norm="softmax", windowing=True)}[variant]
    cfg = TacotronConfig(**kw)
    _, sd = taco_state_dict(None, seed=13, overrides={}, stop_bias=-1e4, cfg=cfg)
    m = build_taco(cfg, sd)
    r = 2
    m.decoder.set_r(r)
    rs = np.random.RandomState(6)
    lens = [17, 5, 40, 2, 29, 12]
    steps = [9, 14, 6, 3, 11, 7]
    batch = np.zeros((len(lens), max(lens)), np.int64)
    for i, L in enumerate(lens):
        batch[i, :L] = rs.randint(1, 129, L)
    dec, post, align, stop = m.inference(torch.from_numpy(batch).cuda(), text_lengths=lens, max_decoder_steps=steps)
    assert list(m.last_steps) == steps
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r, windowing=cfg.windowing, forward_attn=cfg.forward_attn,
                     trans_agent=cfg.trans_agent, forward_attn_mask=cfg.forward_attn_mask, attn_type=cfg.attn_type,
                     attn_K=cfg.attn_K)
    post, align = post.cpu().numpy(), align.cpu().numpy()
    for i, L in enumerate(lens):
        _, p, a, _ = orc.inference(batch[i, :L], r, steps[i])
        M = steps[i] * r
        assert np.abs(post[i, :M] - p).max() <= MEL_TOL
        assert np.abs(align[i, :steps[i], :L] - a).max() <= 1e-5


def test_tacotron2_batch_tiles_shrink_vs_oracle():
    """37 utterances (3 batch tiles) in caller order with the long ones scattered: the decoder
    decodes longest-first and drops to 2 and then 1 batch tile as rows finish; every row must
    still equal its B=1 oracle run, in the caller's order."""
    from oracle.taco_np import TacoOracle
    from tts_amd.spec import TacotronConfig
    _dev()
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=13, overrides={}, stop_bias=-1e4, cfg=cfg)
    m = build_taco(cfg, sd)
    r = 2
    m.decoder.set_r(r)
    rs = np.random.RandomState(9)
    B = 37
    lens = [int(x) for x in rs.randint(2, 24, B)]
    steps = [int(x) for x in rs.randint(2, 9, B)]
    for i in (3, 20, 31):  # a few long rows, not in front
        steps[i] = 41
    for i in (7, 11, 26, 35):
        steps[i] = 23
    T = max(lens)
    batch = np.zeros((B, T), np.int64)
    for i, L in enumerate(lens):
        batch[i, :L] = rs.randint(1, 129, L)
    dec, post, align, stop = m.inference(torch.from_numpy(batch).cuda(), text_lengths=lens, max_decoder_steps=steps)
    assert list(m.last_steps) == steps
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    dec, post, align = dec.cpu().numpy(), post.cpu().numpy(), align.cpu().numpy()
    for i, L in enumerate(lens):
        d, p, a, s = orc.inference(batch[i, :L], r, steps[i])
        M = steps[i] * r
        assert np.abs(dec[i, :M] - d).max() <= MEL_TOL, i
        assert np.abs(post[i, :M] - p).max() <= MEL_TOL, i
        assert np.abs(align[i, :steps[i], :L] - a).max() <= 1e-5, i
        assert not dec[i, M:].any() and not post[i, M:].any()


def test_tacotron2_multichunk_ragged_steps_vs_oracle():
    """B = 70 (two library calls of 64 and 6 rows) with the longest row in the second chunk:
    the joined outputs keep every row's frames and zero padding, and sampled rows of both
    chunks equal their B = 1 oracle runs."""
    from oracle.taco_np import TacoOracle
    from tts_amd.spec import TacotronConfig
    _dev()
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=17, overrides={}, stop_bias=-1e4, cfg=cfg)
    m = build_taco(cfg, sd)
    r = 2
    m.decoder.set_r(r)
    m.decoder.verbose = False
    rs = np.random.RandomState(21)
    B = 70
    lens = [int(x) for x in rs.randint(1, 20, B)]
    steps = [int(x) for x in rs.randint(2, 7, B)]
    steps[66] = 15
    batch = np.zeros((B, max(lens)), np.int64)
    for i, L in enumerate(lens):
        batch[i, :L] = rs.randint(1, 129, L)
    dec, post, align, stop = m.inference(torch.from_numpy(batch).cuda(), text_lengths=lens, max_decoder_steps=steps)
    assert list(m.last_steps) == steps
    S = max(steps)
    assert dec.shape == (B, S * r, 80) and align.shape == (B, S, max(lens)) and stop.shape == (B, S, 1)
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    post, align = post.cpu().numpy(), align.cpu().numpy()
    for i in (0, 31, 63, 64, 66, 69):
        L = lens[i]
        _, p, a, _ = orc.inference(batch[i, :L], r, steps[i])
        M = steps[i] * r
        assert np.abs(post[i, :M] - p).max() <= MEL_TOL, i
        assert np.abs(align[i, :steps[i], :L] - a).max() <= 1e-5, i
    for i in range(B):
        assert not post[i, steps[i] * r:].any() and not align[i, steps[i]:].any()


def test_engine_concurrent_threads_match_sequential():
    """Two host threads share one device context (two Tacotron2 models, so every call re-checks
    and reloads the packed weights, plus the vocoder) on their own streams: every result equals
    the same call made alone."""
    import threading
    from tts_amd.spec import TacotronConfig
    _dev()
    cfg = TacotronConfig()
    models = []
    for seed in (31, 32):
        _, sd = taco_state_dict(None, seed=seed, overrides={}, stop_bias=-1e4, cfg=cfg)
        m = build_taco(cfg, sd)
        m.decoder.set_r(2)
        m.decoder.verbose = False
        models.append(m)
    vcfg, vsd = melgan_state_dict(3)
    voc = build_melgan(vcfg, vsd)
    voc.inference_padding = 0
    rs = np.random.RandomState(3)
    ids = [torch.from_numpy(rs.randint(1, 129, (3, 15))).cuda() for _ in models]

    def run(k):
        _, post, _, _ = models[k].inference(ids[k], max_decoder_steps=[6, 9, 4])
        wav = voc.inference(post.transpose(1, 2).contiguous(), lengths=models[k].last_mel_lengths)
        torch.cuda.current_stream().synchronize()
        return post.cpu(), wav.cpu()

    want = [run(k) for k in (0, 1)]
    got = {0: [], 1: []}
    errs = []

    def worker(k):
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                for _ in range(4):
                    got[k].append(run(k))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for k in (0, 1):
        for post, wav in got[k]:
            assert torch.equal(post, want[k][0]) and torch.equal(wav, want[k][1])


def test_tacotron2_deterministic():
    _dev()
    fx = load_fixture("taco_sigmoid")
    cfg, sd = taco_state_dict(fx, r=2)
    m = build_taco(cfg, sd)
    m.decoder.set_r(2)
    m.decoder.max_decoder_steps = 30
    ids = torch.from_numpy(fx["r2_u2_ids"][None]).cuda()
    a = [t.cpu().numpy() for t in m.inference(ids)]
    b = [t.cpu().numpy() for t in m.inference(ids)]
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_tacotron2_edge_single_token_single_step():
    _dev()
    fx = load_fixture("taco_sigmoid")
    cfg, sd = taco_state_dict(fx, r=2)
    m = build_taco(cfg, sd)
    m.decoder.set_r(2)
    m.decoder.max_decoder_steps = 1
    dec, post, align, stop = m.inference(torch.tensor([[7]], device="cuda"))
    assert dec.shape == (1, 2, 80) and align.shape == (1, 1, 1)
    assert abs(float(align[0, 0, 0]) - 1.0) < 1e-6
    assert list(m.last_status) == [2]


def test_postnet_vs_oracle():
    from oracle.taco_np import TacoOracle
    from tts_amd._lib import get_engine
    from tts_amd.spec import TacotronConfig
    _dev()
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=5, overrides={}, stop_bias=0.0, cfg=cfg)
    m = build_taco(cfg, sd)
    eng = get_engine("cuda:0")
    m._sync(eng)
    rs = np.random.RandomState(9)
    lens = [33, 8, 61]
    M = max(lens)
    dec = np.zeros((3, M, 80), np.float32)
    for i, L in enumerate(lens):
        dec[i, :L] = rs.normal(0, 1, (L, 80))
    out = torch.empty(3, M, 80, device="cuda")
    eng.taco_postnet(torch.from_numpy(dec).cuda(), lens, out)
    out = out.cpu().numpy()
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    for i, L in enumerate(lens):
        assert np.abs(out[i, :L] - orc.postnet(dec[i, :L])).max() <= 1e-4
        assert not out[i, L:].any()


def _synth_models():
    """The seeded Tacotron2-DDC / MB-MelGAN weights behind _synth_files (also the oracle's)."""
    from tts_amd.spec import MelganConfig, TacotronConfig
    from tts_amd.text import symbols
    cfg = TacotronConfig(num_chars=len(symbols))
    _, sd = taco_state_dict(None, seed=21, overrides={}, stop_bias=-1e4, cfg=cfg)
    mcfg, msd = melgan_state_dict(seed=5, cfg=MelganConfig())
    return cfg, sd, mcfg, msd


def _synth_files(tmp_path, with_vocoder=True, stats=False):
    """Checkpoints + configs for Synthesizer. ``stats``: the audio section carries `stats_path`
    (mean-var scaling), as the reference's DDC and MB-MelGAN configs do, pointing at a stats file
    written as TTS/bin/compute_statistics.py writes it."""
    import json as _json
    cfg, sd, mcfg, msd = _synth_models()
    audio = dict(fft_size=1024, win_length=1024, hop_length=256, sample_rate=22050, preemphasis=0.0,
                 ref_level_db=20, power=1.5, griffin_lim_iters=4, num_mels=80, mel_fmin=50.0, mel_fmax=7600.0,
                 spec_gain=1, signal_norm=True, min_level_db=-100, symmetric_norm=True, max_norm=4.0,
                 clip_norm=True)
    if stats:
        rs = np.random.RandomState(11)
        # spec_gain 1: log10 magnitudes, so LJ-like stats are a few units
        st = {"mel_mean": rs.uniform(-3, -1, 80), "mel_std": rs.uniform(0.3, 0.8, 80),
              "linear_mean": rs.uniform(-3, -1, 513), "linear_std": rs.uniform(0.3, 0.8, 513)}
        acfg = {k: v for k, v in audio.items() if k not in ("max_norm", "min_level_db", "symmetric_norm", "clip_norm")}
        audio["stats_path"] = acfg["stats_path"] = str(tmp_path / "scale_stats.npy")
        st["audio_config"] = acfg
        np.save(tmp_path / "scale_stats.npy", st, allow_pickle=True)
    tcfg = {"model": "Tacotron2", "r": 7, "use_phonemes": False, "text_cleaner": "english_cleaners",
            "audio": audio, "attention_norm": "sigmoid", "double_decoder_consistency": True, "ddc_r": 7,
            "prenet_dropout": False, "separate_stopnet": True, "location_attn": True}
    (tmp_path / "tts.json").write_text(_json.dumps(tcfg))
    torch.save({"model": {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, "r": 2},
               str(tmp_path / "tts.pth"))
    conf = {"use_cuda": True, "tts_checkpoint": str(tmp_path / "tts.pth"), "tts_config": str(tmp_path / "tts.json"),
            "tts_speakers": None, "vocoder_checkpoint": None, "vocoder_config": None, "wavernn_lib_path": None}
    if with_vocoder:
        vcfg = {"generator_model": "multiband_melgan_generator", "audio": audio,
                "generator_model_params": {"upsample_factors": list(mcfg.upsample_factors),
                                           "num_res_blocks": mcfg.num_res_blocks}}
        (tmp_path / "voc.json").write_text(_json.dumps(vcfg))
        from tts_amd import MultibandMelganGenerator
        full = MultibandMelganGenerator(in_channels=mcfg.in_channels, out_channels=mcfg.out_channels,
                                        base_channels=mcfg.base_channels, upsample_factors=mcfg.upsample_factors,
                                        num_res_blocks=mcfg.num_res_blocks).state_dict()  # + PQMF buffers
        full.update({k: torch.from_numpy(np.asarray(v)) for k, v in msd.items()})
        torch.save({"model": full}, str(tmp_path / "voc.pth"))
        conf["vocoder_checkpoint"] = str(tmp_path / "voc.pth")
        conf["vocoder_config"] = str(tmp_path / "voc.json")
    return conf


def test_synthesizer_batched_sentences_equal_single(tmp_path):
    """Synthesizer.tts batches all sentences into one Tacotron2 and one vocoder call; each
    sentence must equal its own B=1 synthesis, and tts() must return a readable 16-bit wav."""
    import io
    import scipy.io.wavfile
    from tts_amd.synthesizer import Synthesizer
    _dev()
    synth = Synthesizer(_synth_files(tmp_path))
    synth.tts_model.decoder.max_decoder_steps = 24
    sens = ["Hello world.", "This is a longer test of the batched path, with 2 numbers!", "Short one?"]
    wavs = synth.synthesize_batch(sens)
    assert len(wavs) == 3
    for s, w in zip(sens, wavs):
        ref = synth.synthesize_batch([s])[0]
        assert w.shape == ref.shape == (24 * 2 * 256,)
        assert np.abs(w - ref).max() <= 1e-4
    buf = synth.tts(" ".join(sens))
    sr, x = scipy.io.wavfile.read(io.BytesIO(buf.getvalue()))
    assert sr == 22050 and x.dtype == np.int16 and len(x) >= 3 * 10000


def test_synthesizer_griffin_lim_fallback(tmp_path):
    """No vocoder checkpoint: mel on the GPU, Griffin-Lim on the CPU (config C1's fallback)."""
    from tts_amd.synthesizer import Synthesizer
    _dev()
    synth = Synthesizer(_synth_files(tmp_path, with_vocoder=False))
    synth.tts_model.decoder.max_decoder_steps = 10
    wavs = synth.synthesize_batch(["Griffin and Lim.", "Phase from noise."])
    for w in wavs:
        assert np.isfinite(w).all() and abs(len(w) - 20 * 256) <= 256


def test_synthesizer_mean_var_config_vs_oracle_chain(tmp_path):
    """Synthesizer from configs carrying `stats_path` (TTS/tts/configs/config.json:40,
    vocoder/configs/multiband_melgan_config.json:34), checked against the oracle chain: every
    sentence of synthesize_batch against TacoOracle -> MelganOracle at B = 1 on the same
    text_to_seqvec ids (server/synthesizer.py:144-158), and tts()'s 16-bit wav against the oracle
    waveforms cut by find_endpoint, joined with 10000-sample gaps and scaled as save_wav scales
    (:179-186)."""
    import io
    import scipy.io.wavfile
    from oracle.taco_np import TacoOracle
    from tts_amd.synthesizer import Synthesizer
    from tts_amd.text import text_to_seqvec
    _dev()
    conf = _synth_files(tmp_path, stats=True)
    synth = Synthesizer(conf)
    assert hasattr(synth.ap, "mel_scaler") and synth.ap.signal_norm is True
    steps, r = 24, 2
    synth.tts_model.decoder.max_decoder_steps = steps
    cfg, sd, mcfg, msd = _synth_models()
    to, vo = TacoOracle(sd, cfg.attn_norm, cfg.r), melgan_oracle(mcfg, msd)
    sens = ["Hello world.", "This is a longer test of the batched path, with 2 numbers!", "Short one?"]
    wavs = synth.synthesize_batch(sens)
    refs = []
    for s_, w in zip(sens, wavs):
        ids = text_to_seqvec(s_, synth.tts_config)
        _, p, _, _ = to.inference(ids, r, steps)
        ref = vo.inference(p.T, pad=0).reshape(-1)
        assert w.shape == ref.shape == (steps * r * 256,)
        err = float(np.abs(w - ref).max())
        assert err <= WAV_TOL, (s_, err)
        refs.append(ref)
    buf = synth.tts(" ".join(sens))
    sr, x = scipy.io.wavfile.read(io.BytesIO(buf.getvalue()))
    joined = []
    for ref in refs:
        joined += list(ref[:synth.ap.find_endpoint(ref)]) + [0] * 10000
    joined = np.asarray(joined, np.float32)
    expect = (joined * (32767 / max(0.01, np.max(np.abs(joined))))).astype(np.int16)
    assert sr == 22050 and x.dtype == np.int16 and x.shape == expect.shape
    assert np.abs(x.astype(np.int32) - expect).max() <= 1


def test_synthesis_griffin_lim_mean_var_vs_oracle(tmp_path):
    """synthesis() (tts/utils/synthesis.py:178-262) with a mean-var AudioProcessor: the parsed
    decoder / postnet outputs against the oracle, and the Griffin-Lim waveform (denormalised by the
    mel scaler, audio.py:143-145,241-248, trimmed) against Griffin-Lim of the oracle's postnet
    output under the same random phase."""
    from oracle.taco_np import TacoOracle
    from tts_amd.audio import AudioProcessor
    from tts_amd.factories import load_config
    from tts_amd.synthesis import synthesis, text_to_seqvec
    from tts_amd.synthesizer import Synthesizer
    _dev()
    conf = _synth_files(tmp_path, with_vocoder=False, stats=True)
    model = Synthesizer(conf).tts_model
    steps, r = 10, 2
    model.decoder.max_decoder_steps = steps
    C = load_config(conf["tts_config"])
    ap = AudioProcessor(**C["audio"])
    text = "Hello there, mean and variance."
    np.random.seed(7)
    wav, align, dec, post, stop, _ = synthesis(model, text, C, True, ap, use_griffin_lim=True, do_trim_silence=True)
    cfg, sd, _, _ = _synth_models()
    ids = text_to_seqvec(text, C)
    d, p, a, _ = TacoOracle(sd, cfg.attn_norm, cfg.r).inference(ids, r, steps)
    assert post.shape == p.shape and np.abs(post - p).max() <= MEL_TOL and np.abs(dec - d).max() <= MEL_TOL
    assert (align.argmax(1) == a.argmax(1)).all() and stop.shape[0] == steps
    np.random.seed(7)
    ref = ap.inv_melspectrogram(p.T)
    ref = ref[:ap.find_endpoint(ref)]
    assert wav.shape == ref.shape
    assert np.abs(wav - ref).max() <= 1e-3 * np.abs(ref).max()


def test_synthesizer_gpu_pool_vs_oracle_chain(tmp_path):
    """Synthesizer over a GpuPool (tts_amd.multigpu, one worker process per listed device; device 0
    twice on a one-GPU box): the sentences are sharded by LPT on their token counts and every
    waveform matches the oracle chain. Runs tools/pool_check.py as a fresh child process, since pool
    workers must be started by a process that has not touched the GPU."""
    import subprocess
    import sys
    _dev()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pool_check.py"), str(tmp_path), "0,0"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "pool ok" in r.stdout


def test_mbmelgan_fused_convtranspose_bit_identical(tmp_path):
    """The last upsample's ConvTranspose computed inside the C = 48 ResidualStack kernel
    (resstack_x3.hip CTU = 2, the default) gives the same waveform bits as its own conv_x3 launch
    (TTS_CT_FUSE=0), on a ragged batch: the two modes run in child processes (the switch is read
    once per process) through tools/voc_dump.py."""
    import subprocess
    import sys
    _dev()
    outs = []
    for f in ("0", "1"):
        path = str(tmp_path / f"w{f}.npy")
        env = dict(os.environ, TTS_CT_FUSE=f)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "voc_dump.py"), path], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        outs.append(np.load(path))
    assert outs[0].shape == outs[1].shape and np.array_equal(outs[0], outs[1])


@pytest.mark.gpu
def test_decoder_barrier_block_calibration_bit_identical(tmp_path):
    """The persistent decoder's barrier blocks are picked by timing 16 candidates once per workspace
    (decoder_persist.hip pick_barrier_blocks); where the barrier words live must not change a bit of
    the outputs. Calibrated (with TTS_DIAG_XCC=1 the timings are printed) against the blocks taken in
    order (TTS_BAR_CALIBRATE=0), in child processes (both switches are read once per process),
    through tools/taco_dump.py on 12 LJ-length utterances of the bench model."""
    import subprocess
    import sys
    _dev()
    outs = []
    for cal in ("0", "1"):
        path = str(tmp_path / f"t{cal}.npz")
        env = dict(os.environ, TTS_BAR_CALIBRATE=cal, TTS_DIAG_XCC="1")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "taco_dump.py"), path], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        calibrated = "barrier blocks (us per barrier)" in r.stderr
        assert calibrated == (cal == "1"), r.stderr[-2000:]
        outs.append(np.load(path))
    for k in ("dec", "post", "align", "stop", "steps"):
        assert np.array_equal(outs[0][k], outs[1][k]), k


# --------------------------------------------------------------------- GE2E speaker encoder
@pytest.mark.parametrize("tag,proj", [("proj", True), ("noproj", False)])
def test_ge2e_speaker_encoder_matches_reference(tag, proj):
    """SpeakerEncoder.inference / compute_embedding (TTS/speaker_encoder/model.py:62-88) on the
    persistent 768-unit LSTM: both fixture sequences in ONE batched call with their own lengths."""
    from tts_amd import SpeakerEncoder
    from tts_amd.spec import Ge2eConfig, ge2e_spec
    from tts_amd.weights import synth_state_dict
    _dev()
    fx = load_fixture("ge2e")
    m = SpeakerEncoder(40, 256, 768, 3, proj)
    sd = synth_state_dict(ge2e_spec(Ge2eConfig(use_lstm_with_projection=proj)), int(fx[f"{tag}_seed"]))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    x, x2 = fx["x"][0], fx["x2"][0]
    batch = np.zeros((2, x.shape[0], 40), np.float32)
    batch[0] = x
    batch[1, :len(x2)] = x2
    emb = m.inference(torch.from_numpy(batch).cuda(), lengths=[len(x), len(x2)]).cpu().numpy()
    assert np.abs(emb[0] - fx[f"{tag}_emb"][0]).max() <= 1e-5
    assert np.abs(emb[1] - fx[f"{tag}_emb2"][0]).max() <= 1e-5
    cemb = m.compute_embedding(torch.from_numpy(fx["x"]).cuda()).cpu().numpy()
    assert np.abs(cemb - fx[f"{tag}_cemb"]).max() <= 1e-5


@pytest.mark.parametrize("proj,nl", [(True, 3), (False, 3), (True, 2), (False, 4), (True, 1)])
def test_ge2e_layer_pipeline_matches_per_layer_path(proj, nl):
    """The speaker encoder's layer-pipelined launch (B <= 16, encoder.hip ge2e_pipe_kernel, the
    previous layer's Linear folded into W_ih) against the per-layer launches (B > 16 takes them):
    18 ragged sequences in one call (per-layer) and as two calls of 9 (pipelined), <= 1e-5, for
    1-4 layers (nl x 64 workgroups, one barrier per global step)."""
    from tts_amd import SpeakerEncoder
    from tts_amd.spec import Ge2eConfig, ge2e_spec
    from tts_amd.weights import synth_state_dict
    _dev()
    m = SpeakerEncoder(40, 256, 768, nl, proj)
    sd = synth_state_dict(ge2e_spec(Ge2eConfig(num_lstm_layers=nl, use_lstm_with_projection=proj)), 7)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    rng = np.random.RandomState(3)
    lens = [int(v) for v in rng.randint(20, 97, 18)]
    x = np.zeros((18, max(lens), 40), np.float32)
    for i, n in enumerate(lens):
        x[i, :n] = rng.rand(n, 40).astype(np.float32)
    xt = torch.from_numpy(x).cuda()
    full = m.inference(xt, lengths=lens).cpu().numpy()
    halves = np.concatenate([m.inference(xt[:9], lengths=lens[:9]).cpu().numpy(),
                             m.inference(xt[9:], lengths=lens[9:]).cpu().numpy()])
    assert np.isfinite(full).all()
    assert np.abs(full - halves).max() <= 1e-5


@pytest.mark.parametrize("proj", [True, False])
def test_ge2e_layer_pipeline_short_sequences_vs_oracle(proj):
    """Edge lengths through the layer-pipelined launch: sequences of 1, 2, 3 and 7 frames in one
    call (the pipeline's T + nl - 1 global steps with most layers idle at the ends), every row
    against the numpy oracle (oracle/ge2e_np.py, TTS/speaker_encoder/model.py:62-69)."""
    from oracle.ge2e_np import Ge2eOracle
    from tts_amd import SpeakerEncoder
    from tts_amd.spec import Ge2eConfig, ge2e_spec
    from tts_amd.weights import synth_state_dict
    _dev()
    sd = synth_state_dict(ge2e_spec(Ge2eConfig(use_lstm_with_projection=proj)), 21)
    m = SpeakerEncoder(40, 256, 768, 3, proj)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    go = Ge2eOracle(sd, 3, proj)
    lens = [1, 2, 3, 7]
    rng = np.random.RandomState(4)
    x = np.zeros((4, 7, 40), np.float32)
    for i, n in enumerate(lens):
        x[i, :n] = rng.rand(n, 40).astype(np.float32)
    emb = m.inference(torch.from_numpy(x).cuda(), lengths=lens).cpu().numpy()
    for i, n in enumerate(lens):
        assert np.abs(emb[i] - go.inference(x[i, :n])).max() <= 1e-5, (i, n)


# --------------------------------------------------------------------------------- Glow-TTS
@pytest.mark.parametrize("name,enc", [("glow", "gatedconv"), ("glow_tdsep", "time-depth-separable"),
                                      ("glow_tfm", "transformer")])
def test_glow_tts_matches_reference(name, enc):
    """GlowTts.inference (glow_tts.py:166-193; gated-conv or time-depth-separable encoder, 12 reverse
    flow blocks) with the fixture's prior noise, both utterances in ONE batched call: durations /
    y_lengths and the monotonic path exact, means and mel <= 1e-4."""
    from tts_amd import GlowTts
    from tts_amd.spec import GlowConfig, glow_spec
    from tts_amd.weights import synth_state_dict
    _dev()
    fx = load_fixture(name)
    m = GlowTts(num_chars=GlowConfig().num_chars, encoder_type=enc, use_encoder_prenet=True)
    sd = synth_state_dict(glow_spec(GlowConfig(encoder_type=enc)), int(fx["seed"]))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    ids = [fx["u0_ids"], fx["u1_ids"]]
    T = max(len(x) for x in ids)
    batch = np.zeros((2, T), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    Ty = max(int(fx["u0_ylen"]), int(fx["u1_ylen"]))
    noise = np.zeros((2, 80, Ty), np.float32)
    for i in range(2):
        nz = fx[f"u{i}_noise"]
        noise[i, :, :nz.shape[1]] = nz
    y, _, y_mean, _, attn, logw, _ = m.inference(torch.from_numpy(batch).cuda(), [len(x) for x in ids],
                                                 noise=torch.from_numpy(noise).cuda())
    y, y_mean, attn, logw = y.cpu().numpy(), y_mean.cpu().numpy(), attn.cpu().numpy(), logw.cpu().numpy()
    for i in range(2):
        k = f"u{i}"
        ty, tx = int(fx[k + "_ylen"]), len(ids[i])
        assert m.last_y_lengths[i] == ty
        assert np.abs(logw[i, 0, :tx] - fx[k + "_logw"]).max() <= 1e-5
        assert np.array_equal(attn[i, :ty, :tx], fx[k + "_attn"])
        assert np.abs(y_mean[i, :, :ty] - fx[k + "_ymean"]).max() <= MEL_TOL
        ref = fx[k + "_y"]
        assert np.abs(y[i, :, :ref.shape[1]] - ref).max() <= MEL_TOL
        assert not y[i, :, ref.shape[1]:].any()


def _glow_spk_model(fx):
    from tts_amd import GlowTts
    from tts_amd.spec import GlowConfig, glow_spec
    enc = str(fx["encoder_type"])
    cfg = GlowConfig(encoder_type=enc, num_speakers=int(fx["num_speakers"]), c_in_channels=int(fx["c_in"]))
    sd = synth_state_dict(glow_spec(cfg), int(fx["seed"]))
    m = GlowTts(num_chars=cfg.num_chars, num_speakers=cfg.num_speakers, c_in_channels=cfg.c_in_channels,
                encoder_type=enc, use_encoder_prenet=enc != "gatedconv")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.cuda().eval(), sd


@pytest.mark.parametrize("name", ["glow_spk", "glow_spk_tfm"])
def test_glow_multispeaker_matches_reference(name):
    """Multi-speaker GlowTts with g = speaker ids: the reference's own GlowTts.inference(x,
    x_lengths, g) output (make_golden.py glow_spk: gated-conv encoder, 4 speakers, c_in 36;
    glow_spk_tfm: transformer encoder, 3 speakers, c_in 64), both utterances (speakers 2 and 0) in
    ONE batched call: durations / path exact, means and mel <= 1e-4."""
    _dev()
    fx = load_fixture(name)
    m, _ = _glow_spk_model(fx)
    ids = [fx["u0_ids"], fx["u1_ids"]]
    T = max(len(x) for x in ids)
    batch = np.zeros((2, T), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    Ty = max(int(fx["u0_ylen"]), int(fx["u1_ylen"]))
    noise = np.zeros((2, 80, Ty), np.float32)
    for i in range(2):
        nz = fx[f"u{i}_noise"]
        noise[i, :, :nz.shape[1]] = nz
    g = torch.tensor([int(fx["u0_spk"]), int(fx["u1_spk"])])
    y, _, y_mean, _, attn, logw, _ = m.inference(torch.from_numpy(batch).cuda(), [len(x) for x in ids], g=g,
                                                 noise=torch.from_numpy(noise).cuda())
    y, y_mean, attn, logw = y.cpu().numpy(), y_mean.cpu().numpy(), attn.cpu().numpy(), logw.cpu().numpy()
    for i in range(2):
        k = f"u{i}"
        ty, tx = int(fx[k + "_ylen"]), len(ids[i])
        assert m.last_y_lengths[i] == ty
        assert np.abs(logw[i, 0, :tx] - fx[k + "_logw"]).max() <= 1e-5
        assert np.array_equal(attn[i, :ty, :tx], fx[k + "_attn"])
        assert np.abs(y_mean[i, :, :ty] - fx[k + "_ymean"]).max() <= MEL_TOL
        ref = fx[k + "_y"]
        assert np.abs(y[i, :, :ref.shape[1]] - ref).max() <= MEL_TOL


def test_glow_multispeaker_all_speakers_vs_oracle():
    """One utterance under every speaker of the table in one batch (g = 0..3) against the oracle;
    the speakers give different outputs (the conditioning reaches the flows), and misuse raises as
    the reference does (g on a single-speaker model, no g on a c_in > 0 model, id out of range)."""
    from oracle.glow_np import GlowOracle
    from tts_amd import GlowTts
    _dev()
    fx = load_fixture("glow_spk")
    m, sd = _glow_spk_model(fx)
    orc = GlowOracle(sd)
    ids = fx["u1_ids"]
    outs = [orc.inference(ids, None, 0.0, 1.0, spk=s) for s in range(4)]
    Ty = max(o[4] for o in outs)
    m.noise_scale = 0.0
    x = torch.from_numpy(np.repeat(ids[None], 4, 0)).cuda()
    y, _, ym, _, attn, logw, _ = m.inference(x, [len(ids)] * 4, g=torch.arange(4))
    y, attn = y.cpu().numpy(), attn.cpu().numpy()
    for s, (y_ref, ym_ref, attn_ref, logw_ref, ty) in enumerate(outs):
        assert int(m.last_y_lengths[s]) == ty
        assert np.array_equal(attn[s, :ty], attn_ref)
        assert np.abs(y[s, :, :y_ref.shape[1]] - y_ref).max() <= MEL_TOL
    assert np.abs(outs[0][0][:, :8] - outs[1][0][:, :8]).max() > 1e-2
    with pytest.raises(RuntimeError):
        m.inference(x[:1], [len(ids)])
    with pytest.raises(IndexError):
        m.inference(x[:1], [len(ids)], g=torch.tensor([4]))
    single = GlowTts(num_chars=m.num_chars).cuda().eval()
    with pytest.raises(AttributeError):
        single.inference(x[:1], [len(ids)], g=torch.tensor([0]))


# --------------------------------------------------------------------------------- ParallelWaveGAN
def test_pwgan_matches_reference():
    """ParallelWaveganGenerator.inference with the reference's own prior noise, both fixture mels in
    ONE ragged batch: waveform <= 1e-4 of the reference, zero past each row's length; then the
    weight-norm-folded model gives the same samples."""
    from tts_amd import ParallelWaveganGenerator
    from tts_amd.spec import PwganConfig, pwgan_spec
    from tts_amd.weights import synth_state_dict
    _dev()
    fx = load_fixture("pwgan")
    g = ParallelWaveganGenerator()
    g.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth_state_dict(pwgan_spec(PwganConfig()), int(fx["seed"])).items()})
    g = g.cuda().eval()
    Ms = (5, 11)
    M = max(Ms)
    mel = np.zeros((2, 80, M), np.float32)
    T = 256 * (M + 4)
    noise = np.zeros((2, 1, T), np.float32)
    for i, m in enumerate(Ms):
        mel[i, :, :m] = fx[f"M{m}_mel"][0]
        noise[i, 0, :256 * (m + 4)] = fx[f"M{m}_noise"][0, 0]
    outs = []
    for fold in (False, True):
        if fold:
            g.remove_weight_norm()
        y = g.inference(torch.from_numpy(mel).cuda(), lengths=list(Ms), noise=torch.from_numpy(noise).cuda())
        y = y.cpu().numpy()
        for i, m in enumerate(Ms):
            ref = fx[f"M{m}_wav"][0, 0]
            assert np.abs(y[i, 0, :len(ref)] - ref).max() <= 1e-4
            assert not y[i, 0, len(ref):].any()
        outs.append(y)
    assert np.abs(outs[0] - outs[1]).max() <= 1e-5


def test_synthesizer_glow_tts_and_pwgan(tmp_path):
    """Config C4 through the server path: model "glow_tts" + "parallel_wavegan_generator"
    (setup_model / setup_generator), all sentences in one Glow call and one PWGAN call; each
    waveform is hop * 2 * floor(y_length / 2) samples (a B = 1 reference call's length)."""
    import json as _json
    from tts_amd import GlowTts, ParallelWaveganGenerator
    from tts_amd.spec import GlowConfig, PwganConfig, glow_spec, pwgan_spec
    from tts_amd.synthesizer import Synthesizer
    from tts_amd.text import symbols
    from tts_amd.weights import synth_state_dict
    _dev()
    conf = _synth_files(tmp_path, with_vocoder=False)
    tcfg = _json.loads((tmp_path / "tts.json").read_text())
    tcfg.update({"model": "glow_tts", "encoder_type": "gatedconv"})
    (tmp_path / "glow.json").write_text(_json.dumps(tcfg))
    gsd = synth_state_dict(glow_spec(GlowConfig(num_chars=len(symbols))), 23)
    torch.save({"model": {k: torch.from_numpy(v) for k, v in gsd.items()}}, str(tmp_path / "glow.pth"))
    vcfg = {"generator_model": "parallel_wavegan_generator", "audio": tcfg["audio"],
            "generator_model_params": {"upsample_factors": [4, 4, 4, 4], "stacks": 3, "num_res_blocks": 30}}
    (tmp_path / "pwg.json").write_text(_json.dumps(vcfg))
    psd = synth_state_dict(pwgan_spec(PwganConfig()), 31)
    torch.save({"model": {k: torch.from_numpy(v) for k, v in psd.items()}}, str(tmp_path / "pwg.pth"))
    conf.update({"tts_checkpoint": str(tmp_path / "glow.pth"), "tts_config": str(tmp_path / "glow.json"),
                 "vocoder_checkpoint": str(tmp_path / "pwg.pth"), "vocoder_config": str(tmp_path / "pwg.json")})
    synth = Synthesizer(conf)
    assert isinstance(synth.tts_model, GlowTts) and isinstance(synth.vocoder_model, ParallelWaveganGenerator)
    sens = ["Hello world.", "A longer sentence for the flow decoder!"]
    wavs = synth.synthesize_batch(sens)
    ylens = synth.tts_model.last_y_lengths
    for w, yl in zip(wavs, ylens):
        assert w.shape == (256 * 2 * (int(yl) // 2),) and np.isfinite(w).all() and np.abs(w).max() > 0


def test_pwgan_persistent_kernel_bit_identical(tmp_path):
    """The persistent, weight-resident residual-block kernel (pw_layer_x3p_kernel, the default) gives
    the same waveform bits as the per-tile kernel (TTS_PWGAN_TILE=1) on a ragged 3-utterance LJ
    batch with one seeded prior; the two modes run in child processes (tools/pwgan_bench.py --dump)."""
    import subprocess
    import sys
    _dev()
    outs = []
    for f in ("0", "1"):
        path = str(tmp_path / f"p{f}.npy")
        env = dict(os.environ, TTS_PWGAN_TILE=f)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pwgan_bench.py"), "--batch", "3", "--steps", "1",
                            "--warmup", "0", "--dump", path], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        outs.append(np.load(path))
    assert outs[0].shape == outs[1].shape and np.array_equal(outs[0], outs[1])


def test_pwgan_inference_padding_zero_vs_oracle():
    """inference_padding = 0 (what Synthesizer sets, server/synthesizer.py:86) against the fp32
    oracle on the fixture weights and mel (parity pinned through the oracle, <= 2e-6 of the reference)."""
    from oracle.pwgan_np import PwganOracle
    from tts_amd import ParallelWaveganGenerator
    from tts_amd.spec import PwganConfig, pwgan_spec
    _dev()
    fx = load_fixture("pwgan")
    cfg = PwganConfig(inference_padding=0)
    sd = synth_state_dict(pwgan_spec(PwganConfig()), int(fx["seed"]))
    g = ParallelWaveganGenerator(inference_padding=0)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    g = g.cuda().eval()
    mel = fx["M5_mel"]
    noise = np.random.RandomState(3).randn(1, 1, 5 * 256).astype(np.float32)
    y = g.inference(torch.from_numpy(mel).cuda(), noise=torch.from_numpy(noise).cuda()).cpu().numpy()[0, 0]
    ref = PwganOracle(sd, cfg).inference(mel[0], noise[0, 0])
    assert y.shape == ref.shape == (5 * 256,)
    assert np.abs(y - ref).max() <= 1e-4


def test_pwgan_split_f16_equals_fp32_path_and_oracle():
    """The split-f16 residual-block kernel (pw_layer_x3_kernel, the default) against the fp32-MFMA
    kernel and the oracle on a ragged 2-row batch long enough for every dilation (up to 512): both
    within 1e-4 of the oracle, the split path's error at most twice the fp32 path's plus 2e-6, no
    range fallback; an input scaled past the f16 range re-runs in fp32, bit-identical."""
    from oracle.pwgan_np import PwganOracle
    from tts_amd import ParallelWaveganGenerator
    from tts_amd.spec import PwganConfig, pwgan_spec
    _dev()
    fx = load_fixture("pwgan")
    cfg = PwganConfig(inference_padding=0)
    sd = synth_state_dict(pwgan_spec(PwganConfig()), int(fx["seed"]))
    g = ParallelWaveganGenerator(inference_padding=0)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    g = g.cuda().eval()
    rs = np.random.RandomState(21)
    lens = [9, 4]
    mel = np.zeros((2, 80, 9), np.float32)
    for i, L in enumerate(lens):
        mel[i, :, :L] = rs.uniform(-1, 1, (80, L))
    noise = rs.randn(2, 1, 9 * 256).astype(np.float32)
    m, n = torch.from_numpy(mel).cuda(), torch.from_numpy(noise).cuda()
    eng = _gemm("f32")
    try:
        y32 = g.inference(m, lengths=lens, noise=n).cpu().numpy()
        big32 = g.inference(m * 1e6, lengths=lens, noise=n).cpu().numpy()
    finally:
        eng = _gemm("x3")
    n0 = eng.gemm_mode()[1]
    y16 = g.inference(m, lengths=lens, noise=n).cpu().numpy()
    assert eng.gemm_mode() == ("x3", n0)
    orc = PwganOracle(sd, cfg)
    e16 = e32 = 0.0
    for i, L in enumerate(lens):
        ref = orc.inference(mel[i, :, :L], noise[i, 0, :L * 256])
        e16 = max(e16, float(np.abs(y16[i, 0, :L * 256] - ref).max()))
        e32 = max(e32, float(np.abs(y32[i, 0, :L * 256] - ref).max()))
        assert not y16[i, 0, L * 256:].any()
    print(f"PWGAN waveform error vs oracle: split-f16 {e16:.2e}, fp32 {e32:.2e}")
    assert e16 <= 1e-4 and e32 <= 1e-4
    assert e16 <= 2 * e32 + 2e-6
    big16 = g.inference(m * 1e6, lengths=lens, noise=n).cpu().numpy()
    assert eng.gemm_mode()[1] == n0 + 1
    assert np.array_equal(big16, big32, equal_nan=True)


def test_glow_length_and_noise_scale_vs_oracle():
    """GlowTts.length_scale / noise_scale (glow_tts.py:172-186) away from their defaults, against the
    oracle: y_lengths and the path exact, mel <= 1e-4."""
    from oracle.glow_np import GlowOracle
    from tts_amd import GlowTts
    from tts_amd.spec import GlowConfig, glow_spec
    _dev()
    fx = load_fixture("glow")
    sd = synth_state_dict(glow_spec(GlowConfig()), int(fx["seed"]))
    m = GlowTts(num_chars=GlowConfig().num_chars)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    ids = fx["u1_ids"]
    orc = GlowOracle(sd)
    # durations are ceil((exp(logw) - 1) * length_scale): take a scale that leaves every token's
    # value >= 1e-3 away from an integer, so 1e-6-level differences in logw cannot flip a ceil
    _, logw = orc.encode(ids)
    w = np.exp(logw.astype(np.float64)) - 1
    ls = next(x for x in (1.7, 1.45, 1.3, 0.85, 1.15) if np.abs(w * x - np.round(w * x)).min() > 1e-3)
    m.length_scale, m.noise_scale = ls, 0.4
    _, _, _, _, Ty0 = orc.inference(ids, None, 0.4, ls)
    noise = np.random.RandomState(5).randn(1, 80, Ty0).astype(np.float32)
    y_ref, ym_ref, attn_ref, logw_ref, Ty = orc.inference(ids, noise[0], 0.4, ls)
    y, _, ym, _, attn, _, _ = m.inference(torch.from_numpy(ids[None]).cuda(), [len(ids)],
                                          noise=torch.from_numpy(noise).cuda())
    assert int(m.last_y_lengths[0]) == Ty
    assert np.array_equal(attn.cpu().numpy()[0], attn_ref)
    assert np.abs(y.cpu().numpy()[0] - y_ref).max() <= 1e-4


def test_synthesizer_multispeaker(tmp_path):
    """tts_speakers mapping (synthesizer.py:62-67) -> num_speakers; tts(text, speaker_id) decodes every
    sentence with that speaker's learned embedding: each equals the model's own B = 1 call."""
    import json as _json
    from tts_amd.spec import TacotronConfig
    from tts_amd.synthesizer import Synthesizer
    from tts_amd.text import symbols
    _dev()
    conf = _synth_files(tmp_path)
    cfg = TacotronConfig(num_chars=len(symbols), num_speakers=4)
    _, sd = taco_state_dict(None, seed=21, overrides={}, stop_bias=-1e4, cfg=cfg)
    torch.save({"model": {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, "r": 2},
               str(tmp_path / "tts_ms.pth"))
    (tmp_path / "speakers.json").write_text(_json.dumps({f"spk{i}": i for i in range(4)}))
    conf.update({"tts_checkpoint": str(tmp_path / "tts_ms.pth"), "tts_speakers": str(tmp_path)})
    synth = Synthesizer(conf)
    assert synth.tts_model.num_speakers == 4
    synth.tts_model.decoder.max_decoder_steps = 12
    sens = ["Hello world.", "Speaker two speaks here."]
    wavs = synth.synthesize_batch(sens, speaker_id=2)
    for s_, w in zip(sens, wavs):
        ref = synth.synthesize_batch([s_], speaker_id=2)[0]
        assert w.shape == ref.shape and np.abs(w - ref).max() <= 1e-4
    other = synth.synthesize_batch(sens[:1], speaker_id=0)[0]
    assert np.abs(other - wavs[0]).max() > 1e-3


def test_synthesis_notebook_surface(tmp_path):
    """synthesis(model, text, CONFIG, use_cuda, ap, ...) (tts/utils/synthesis.py:178-262), the
    notebooks' entry: outputs are the model's own B = 1 inference, parsed as the reference parses
    them; Griffin-Lim on request; truncated=True raises as the reference does."""
    from tts_amd.audio import AudioProcessor
    from tts_amd.factories import load_config
    from tts_amd.synthesis import synthesis, text_to_seqvec
    from tts_amd.synthesizer import Synthesizer
    _dev()
    conf = _synth_files(tmp_path, with_vocoder=False)
    synth = Synthesizer(conf)
    model = synth.tts_model
    model.decoder.max_decoder_steps = 10
    C = load_config(conf["tts_config"])
    ap = AudioProcessor(**C["audio"])
    wav, align, dec, post, stop, inputs = synthesis(model, "Hello there.", C, True, ap, use_griffin_lim=True)
    ids = text_to_seqvec("Hello there.", C)
    d2, p2, a2, s2 = model.inference(torch.from_numpy(ids[None].astype(np.int64)).cuda())
    assert np.array_equal(post, p2[0].cpu().numpy()) and np.array_equal(dec, d2[0].cpu().numpy())
    assert align.shape == a2[0].shape and stop.shape == s2[0].shape
    assert wav is not None and np.isfinite(wav).all() and tuple(inputs.shape) == (1, len(ids))
    with pytest.raises(AttributeError):
        synthesis(model, "Hello there.", C, True, ap, truncated=True)


def test_synthesize_cli(tmp_path):
    """python -m tts_amd.synthesize (TTS/bin/synthesize.py): Tacotron2-DDC + MB-MelGAN from
    checkpoint files; the 16-bit wav is named after the text as the reference names it."""
    import scipy.io.wavfile
    from tts_amd.synthesize import main
    _dev()
    conf = _synth_files(tmp_path)
    out = main(["Hi there, MI355X.", conf["tts_config"], conf["tts_checkpoint"], str(tmp_path),
                "--vocoder_path", conf["vocoder_checkpoint"], "--vocoder_config_path", conf["vocoder_config"]])
    assert os.path.basename(out) == "Hi_there_MI355X.wav"
    sr, x = scipy.io.wavfile.read(out)
    assert sr == 22050 and len(x) > 0


def test_pwgan_single_frame_vs_oracle():
    """Edge: a one-frame mel (5 frames after the replicate padding: 1280 samples, ten 128-sample
    tiles of the residual-block grid) against the oracle."""
    from oracle.pwgan_np import PwganOracle
    from tts_amd import ParallelWaveganGenerator
    from tts_amd.spec import PwganConfig, pwgan_spec
    _dev()
    fx = load_fixture("pwgan")
    sd = synth_state_dict(pwgan_spec(PwganConfig()), int(fx["seed"]))
    g = ParallelWaveganGenerator()
    g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    g = g.cuda().eval()
    mel = fx["M5_mel"][:, :, :1]
    noise = np.random.RandomState(7).randn(1, 1, 5 * 256).astype(np.float32)
    y = g.inference(torch.from_numpy(mel).cuda(), noise=torch.from_numpy(noise).cuda()).cpu().numpy()[0, 0]
    ref = PwganOracle(sd, PwganConfig()).inference(mel[0], noise[0, 0])
    assert y.shape == ref.shape == (5 * 256,)
    assert np.abs(y - ref).max() <= 1e-4


def test_glow_short_utterances_vs_oracle():
    """Edge: two-token and three-token utterances batched with a long one (ragged T_x, small T_y)."""
    from oracle.glow_np import GlowOracle
    from tts_amd import GlowTts
    from tts_amd.spec import GlowConfig, glow_spec
    _dev()
    fx = load_fixture("glow")
    sd = synth_state_dict(glow_spec(GlowConfig()), int(fx["seed"]))
    m = GlowTts(num_chars=GlowConfig().num_chars)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    orc = GlowOracle(sd)
    long_ids = fx["u1_ids"]

    def short(n):  # the first n-token window whose T_y >= 2 (T_y < 2 leaves the reference's squeeze empty)
        for s0 in range(len(long_ids) - n):
            if orc.inference(long_ids[s0:s0 + n], None, 0.0, 1.0)[4] >= 2:
                return long_ids[s0:s0 + n]
        raise AssertionError("no usable window")
    cands = [short(2), short(3), long_ids]
    outs = [orc.inference(x, None, 0.0, 1.0) for x in cands]
    Ty = max(o[4] for o in outs)
    batch = np.zeros((3, len(long_ids)), np.int64)
    for i, x in enumerate(cands):
        batch[i, :len(x)] = x
    m.noise_scale = 0.0
    y, _, ym, _, attn, _, _ = m.inference(torch.from_numpy(batch).cuda(), [len(x) for x in cands],
                                          noise=torch.zeros(3, 80, Ty).cuda())
    y = y.cpu().numpy()
    for i, (yr, ymr, ar, _, ty) in enumerate(outs):
        assert int(m.last_y_lengths[i]) == ty
        assert np.array_equal(attn.cpu().numpy()[i, :ty, :len(cands[i])], ar)
        assert np.abs(y[i, :, :yr.shape[1]] - yr).max() <= 1e-4


def test_bench_workload_full_size_vs_oracle():
    """The headline workload at its full size (bench.py: 32 LJ-profile utterances in one batch,
    r = 2, forced lengths of up to 429 decoder steps, the bench's own weights), every utterance
    checked against the oracle run at B = 1, like the reference CPU path: mel L-inf within 1e-4
    (north_star), alignment argmax indices identical; and EVERY row of the bench's own batched
    MB-MelGAN call (per-row lengths, read in place from the frame-major postnet output) within
    WAV_TOL of the oracle chain's waveform (oracle mel -> oracle vocoder, multiband_melgan_generator.py:32-39),
    zero past its length. Measured: mel error ~1e-6 at 429 steps."""
    import bench
    from oracle.melgan_np import MelganOracle
    from oracle.taco_np import TacoOracle
    from tts_amd.pqmf import pqmf_filters
    from tts_amd.spec import melgan_layers
    from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids
    dev = _dev()
    taco, tsd, voc, vsd, tcfg, vcfg = bench.build_models(dev)
    r = 2
    taco.decoder.set_r(r)
    taco.decoder.verbose = False
    T_prof, M_prof = lj_profile()
    ids = synthetic_ids(T_prof)
    steps = forced_steps(M_prof, r)
    batch, lens = pad_batch(ids)
    mlens = [S * r for S in steps]
    with torch.no_grad():
        dec, post, align, stop = taco.inference(torch.from_numpy(batch).to(dev), text_lengths=lens,
                                                max_decoder_steps=steps)
        assert list(taco.last_steps) == list(steps)
        wavb = voc.inference(post.transpose(1, 2), lengths=taco.last_mel_lengths).cpu().numpy()
    post, align = post.cpu().numpy(), align.cpu().numpy()
    to = TacoOracle(tsd, tcfg.attn_norm, tcfg.r)
    vo = MelganOracle(vsd, melgan_layers(vcfg), pqmf_filters()[1])
    worst = worst_w = 0.0
    for i in range(len(ids)):
        L, S = len(ids[i]), steps[i]
        _, p, a, _ = to.inference(ids[i], r, S)
        M = S * r
        err = float(np.abs(post[i, :M] - p).max())
        worst = max(worst, err)
        assert err <= MEL_TOL, (i, L, S, err)
        assert (align[i, :S, :L].argmax(1) == a.argmax(1)).all(), i
        ref = vo.inference(p.T, pad=0).reshape(-1)
        assert ref.size == 256 * mlens[i]
        werr = float(np.abs(wavb[i, 0, :ref.size] - ref).max())
        worst_w = max(worst_w, werr)
        assert werr <= WAV_TOL, (i, werr)
        assert not wavb[i, 0, ref.size:].any(), i
    print(f"32 utterances, worst mel error {worst:.2e}, worst waveform error {worst_w:.2e}")


@pytest.mark.parametrize("pad", [0, 2])
def test_fused_taco_mbmelgan_equals_two_calls(pad):
    """Tacotron2.inference_vocoded (tts_taco_mbmelgan_infer: the decode's lengths handed to the
    vocoder inside the library) against the reference's call pair, Tacotron2.inference then
    MultibandMelganGenerator.inference(postnet.transpose(1, 2), lengths) (server/synthesizer.py:
    150-159): every output bit-identical, ragged forced lengths over the 32-row LJ batch (steps cut
    to a quarter), inference padding 0 and 2; the per-row lengths on the model agree too."""
    import bench
    from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids
    dev = _dev()
    taco, tsd, voc, vsd, tcfg, vcfg = bench.build_models(dev)
    voc.inference_padding = pad
    taco.decoder.set_r(2)
    taco.decoder.verbose = False
    T_prof, M_prof = lj_profile()
    ids = synthetic_ids(T_prof)
    steps = [max(3, s_ // 4) for s_ in forced_steps(M_prof, 2)]
    batch, lens = pad_batch(ids)
    x = torch.from_numpy(batch).to(dev)
    with torch.no_grad():
        a = taco.inference(x, text_lengths=lens, max_decoder_steps=steps)
        ml = taco.last_mel_lengths.copy()
        wa = voc.inference(a[1].transpose(1, 2), lengths=ml)
        b = taco.inference_vocoded(x, voc, text_lengths=lens, max_decoder_steps=steps)
    assert list(taco.last_mel_lengths) == list(ml) == [2 * s_ for s_ in steps]
    for u, v in zip(a + (wa,), b):
        assert u.shape == v.shape and torch.equal(u, v)
    assert wa.shape[-1] == voc.hop * (max(ml) + 2 * pad)


def test_mbmelgan_beside_concurrent_bilstm_bit_identical():
    """MB-MelGAN.inference of one library context on its own stream while another context runs
    persistent encoder BiLSTM launches: every waveform bit-identical to the same call run alone.
    Before the PQMF synthesis loop's FMAs were kept out of v_pk_fma_f32 (melgan_out.hip,
    fma_nopk), 13 of 80 such trials had runs of 16 wrong samples in output phases 0 / 2
    (tools/race_probe.py, profiles/r06/v26_pqmf_opsel.txt); 24 trials would have caught it
    with probability ~0.99."""
    from concurrent.futures import ThreadPoolExecutor

    import bench
    from tts_amd._lib import Engine, get_engine
    from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids
    dev = _dev()
    taco, tsd, voc, vsd, tcfg, vcfg = bench.build_models(dev)
    taco.decoder.set_r(2)
    taco.decoder.verbose = False
    T_prof, M_prof = lj_profile()
    batch, lens = pad_batch(synthetic_ids(T_prof))
    x = torch.from_numpy(batch).to(dev)
    with torch.no_grad():
        _, post, _, _ = taco.inference(x, text_lengths=lens, max_decoder_steps=forced_steps(M_prof, 2))
    ml = np.asarray(taco.last_mel_lengths, np.int64)
    c = post.transpose(1, 2).contiguous()
    B, _, M = c.shape
    engB = Engine(0)
    try:
        voc._sync(engB)
        ea = get_engine(dev)
        sV = torch.cuda.Stream(dev)

        def voc_call():
            with torch.cuda.stream(sV):
                w = torch.full((B, 1, voc.hop * M), float("nan"), device=dev)
                engB.melgan_infer(c, ml, 0, w)
                sV.synchronize()
            return w

        ref = voc_call().clone()
        assert not torch.isnan(ref).any()
        eo = torch.empty(x.shape[0], x.shape[1], 512, device=dev)
        bad = []
        with ThreadPoolExecutor(1) as ex:
            for trial in range(24):
                torch.cuda.synchronize()
                fut = ex.submit(voc_call)
                with ea.lock:
                    for _ in range(6):
                        ea.taco_encoder(x, lens, eo)
                w = fut.result()
                torch.cuda.synchronize()
                if not torch.equal(w, ref):
                    bad.append((trial, int((w != ref).sum())))
        assert not bad, f"waveforms differ beside the BiLSTM (trial, samples): {bad}"
    finally:
        engB.close()


def test_fused_submit_pipelined_and_short_decode():
    """The fused call's two halves (tts_taco_mbmelgan_submit / _finish) with the host one batch
    ahead, as bench.py times it: two batches with different ragged forced lengths submitted back to
    back, then both finished; each batch bit-identical to its two-call form. Then the vocoder
    launched on device-side lengths below the S_cap bound (S_cap = max steps + 7: the waveform rows
    are packed back to hop (M + 2 pad) samples apart), blocking and submitted; one utterance at
    padding 2 against its two calls, and an unknown ticket refused; and a decode whose
    rows stop at step 2 (stop threshold -1, r = 1: 2 mel frames, shorter than ReflectionPad1d(3)
    allows) fails the call with the vocoder's length message, the context usable afterwards."""
    import bench
    from tts_amd._lib import get_engine
    from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids
    dev = _dev()
    taco, tsd, voc, vsd, tcfg, vcfg = bench.build_models(dev)
    taco.decoder.set_r(2)
    taco.decoder.verbose = False
    T_prof, M_prof = lj_profile()
    ids = synthetic_ids(T_prof)
    batch, lens = pad_batch(ids)
    x = torch.from_numpy(batch).to(dev)
    full = forced_steps(M_prof, 2)
    steps_a = [max(3, s_ // 5) for s_ in full]
    steps_b = [max(3, s_ // 7) for s_ in full][::-1]

    def two_calls(steps):
        a = taco.inference(x, text_lengths=lens, max_decoder_steps=steps)
        return a + (voc.inference(a[1].transpose(1, 2), lengths=taco.last_mel_lengths.copy()),)

    with torch.no_grad():
        ref_a, ref_b = two_calls(steps_a), two_calls(steps_b)
        fa = taco.inference_vocoded_submit(x, voc, text_lengths=lens, max_decoder_steps=steps_a)
        fb = taco.inference_vocoded_submit(x, voc, text_lengths=lens, max_decoder_steps=steps_b)
        got_a, got_b = fa.result(), fb.result()
        assert fa.result() is not None  # finishing twice is harmless
    for ref, got in ((ref_a, got_a), (ref_b, got_b)):
        for u, v in zip(ref, got):
            assert u.shape == v.shape and torch.equal(u, v)

    # S_cap above the decoded steps: rows packed after the vocoder, blocking and submitted
    eng = get_engine(dev)
    Tn, B, r, pad = int(max(lens)), len(ids), 2, int(voc.inference_padding)
    S_cap = max(steps_a) + 7
    sub = x[:, :Tn].contiguous()
    for submit in (False, True):
        dec, post, align, stop = taco._out_tensors(B, S_cap, r, Tn, dev)
        wbuf = torch.full((B * voc.hop * (S_cap * r + 2 * pad),), float("nan"), device=dev)
        args = (sub, lens, r, np.asarray(steps_a), S_cap, taco.decoder.stop_threshold, dec, post, align, stop, pad, wbuf)
        with eng.lock:
            if submit:
                st, _, ticket = eng.taco_mbmelgan_submit(*args)
                eng.taco_mbmelgan_finish(ticket, dev)
            else:
                st, _ = eng.taco_mbmelgan_infer(*args)
        assert list(st) == steps_a
        L = voc.hop * (max(steps_a) * r + 2 * pad)
        assert torch.equal(wbuf[:B * L].view(B, 1, L), ref_a[4])
        assert torch.equal(post[:, :max(steps_a) * r], ref_a[1])

    # one utterance, inference padding 2, S_cap above its steps; a ticket never handed out is refused
    voc.inference_padding = 2
    try:
        x1 = x[3:4, :lens[3]].contiguous()
        with torch.no_grad():
            a1 = taco.inference(x1, max_decoder_steps=[steps_a[3]])
            w1 = voc.inference(a1[1].transpose(1, 2), lengths=taco.last_mel_lengths.copy())
        S1 = steps_a[3] + 5
        dec, post, align, stop = taco._out_tensors(1, S1, r, lens[3], dev)
        wbuf = torch.full((voc.hop * (S1 * r + 4),), float("nan"), device=dev)
        with eng.lock:
            st, _, ticket = eng.taco_mbmelgan_submit(x1, [lens[3]], r, np.asarray([steps_a[3]]), S1,
                                                     taco.decoder.stop_threshold, dec, post, align, stop, 2, wbuf)
            eng.taco_mbmelgan_finish(ticket, dev)
            with pytest.raises(RuntimeError, match="unknown ticket"):
                eng.taco_mbmelgan_finish(ticket + 1000, dev)
        L1 = voc.hop * (steps_a[3] * r + 4)
        assert list(st) == [steps_a[3]] and torch.equal(wbuf[:L1].view(1, 1, L1), w1)
    finally:
        voc.inference_padding = 0

    # rows that stop at step 2 at r = 1: 2 frames, below the vocoder's reflection pad
    taco.decoder.set_r(1)
    thr = taco.decoder.stop_threshold
    taco.decoder.stop_threshold = -1.0
    try:
        with torch.no_grad(), pytest.raises(RuntimeError, match="shorter than the vocoder"):
            taco.inference_vocoded(x, voc, text_lengths=lens, max_decoder_steps=[10] * B)
    finally:
        taco.decoder.stop_threshold = thr
        taco.decoder.set_r(2)
    with torch.no_grad():
        again = taco.inference_vocoded(x, voc, text_lengths=lens, max_decoder_steps=steps_a)
    for u, v in zip(ref_a, again):
        assert torch.equal(u, v)


def test_fused_submit_b64_equals_two_calls():
    """The fused submission at the largest batch one decode takes (64 rows: the LJ profile twice,
    MT = 4 batch tiles; the vocoder's persistent kernels count their tiles from 64 device-side
    lengths): every output bit-identical to Tacotron2.inference + MultibandMelganGenerator.inference."""
    import bench
    from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids
    dev = _dev()
    taco, tsd, voc, vsd, tcfg, vcfg = bench.build_models(dev)
    taco.decoder.set_r(2)
    taco.decoder.verbose = False
    T_prof, M_prof = lj_profile()
    ids = synthetic_ids(T_prof) * 2
    steps = [max(3, s_ // 6) for s_ in forced_steps(M_prof, 2)] * 2
    steps = steps[32:] + steps[:32][::-1]
    batch, lens = pad_batch(ids)
    x = torch.from_numpy(batch).to(dev)
    with torch.no_grad():
        a = taco.inference(x, text_lengths=lens, max_decoder_steps=steps)
        wa = voc.inference(a[1].transpose(1, 2), lengths=taco.last_mel_lengths.copy())
        b = taco.inference_vocoded_submit(x, voc, text_lengths=lens, max_decoder_steps=steps).result()
    assert len(b[0]) == 64
    for u, v in zip(a + (wa,), b):
        assert u.shape == v.shape and torch.equal(u, v)


def test_bench_workload_full_size_r1_vs_oracle():
    """The bench line's r = 1 run at its full length (bench.py `r1`: the same 32 LJ-profile
    utterances, forced lengths of up to 857 decoder steps, one frame per step as the
    Decoder.inference loop of layers/tacotron2.py:354-369 runs it at r = 1), every utterance against
    the oracle at B = 1: mel L-inf within 1e-4 (north_star), every step's alignment argmax identical,
    and the two longest rows' MB-MelGAN waveforms (from the bench's batched vocoder call) within
    WAV_TOL of the oracle chain."""
    import bench
    from oracle.melgan_np import MelganOracle
    from oracle.taco_np import TacoOracle
    from tts_amd.pqmf import pqmf_filters
    from tts_amd.spec import melgan_layers
    from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids
    dev = _dev()
    taco, tsd, voc, vsd, tcfg, vcfg = bench.build_models(dev)
    r = 1
    taco.decoder.set_r(r)
    taco.decoder.verbose = False
    T_prof, M_prof = lj_profile()
    ids = synthetic_ids(T_prof)
    steps = forced_steps(M_prof, r)
    assert max(steps) >= 850
    batch, lens = pad_batch(ids)
    with torch.no_grad():
        _, post, align, _ = taco.inference(torch.from_numpy(batch).to(dev), text_lengths=lens,
                                           max_decoder_steps=steps)
        assert list(taco.last_steps) == list(steps)
        wavb = voc.inference(post.transpose(1, 2), lengths=taco.last_mel_lengths).cpu().numpy()
    taco.decoder.set_r(tcfg.r)
    post, align = post.cpu().numpy(), align.cpu().numpy()
    to = TacoOracle(tsd, tcfg.attn_norm, tcfg.r)
    longest = set(np.argsort(steps)[-2:].tolist())
    vo = MelganOracle(vsd, melgan_layers(vcfg), pqmf_filters()[1])
    worst = worst_w = 0.0
    for i in range(len(ids)):
        L, S = len(ids[i]), steps[i]
        _, p, a, _ = to.inference(ids[i], r, S)
        assert p.shape[0] == S
        err = float(np.abs(post[i, :S] - p).max())
        worst = max(worst, err)
        assert err <= MEL_TOL, (i, L, S, err)
        assert (align[i, :S, :L].argmax(1) == a.argmax(1)).all(), i
        if i in longest:
            ref = vo.inference(p.T, pad=0).reshape(-1)
            werr = float(np.abs(wavb[i, 0, :ref.size] - ref).max())
            worst_w = max(worst_w, werr)
            assert werr <= WAV_TOL, (i, werr)
            assert not wavb[i, 0, ref.size:].any(), i
    print(f"r=1, 32 utterances ({sum(steps)} row-steps, {max(steps)} max), worst mel error {worst:.2e}, "
          f"worst waveform error (2 longest) {worst_w:.2e}")


def test_glow_lj_batch_full_size_vs_oracle():
    """Glow-TTS on tools/glow_bench.py's workload at full size (32 LJ-profile utterances, 3346
    tokens, ~19 k frames, seed-3 weights), every utterance against the oracle at B = 1: y_lengths and
    the path exact, mel <= 1e-4. length_scale is taken near the bench's calibrated value where every
    token's ceil((exp(logw) - 1) * ls) argument is >= 2e-5 away from an integer, so the ~1e-6
    differences in logw cannot flip a duration (the reference itself is only defined up to that)."""
    from oracle.glow_np import GlowOracle
    from tts_amd import GlowTts
    from tts_amd.spec import GlowConfig, glow_spec
    from tts_amd.workload import lj_profile, pad_batch, synthetic_ids
    _dev()
    cfg = GlowConfig()
    sd = synth_state_dict(glow_spec(cfg), 3)
    m = GlowTts(num_chars=cfg.num_chars)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    T, M = lj_profile()
    ids = synthetic_ids(T)
    orc = GlowOracle(sd)
    w = [np.exp(orc.encode(x)[1].astype(np.float64)).reshape(-1) - 1 for x in ids]
    base = sum(M) / float(sum(np.ceil(np.maximum(v, 0)).sum() for v in w))
    ls = next(s for s in base * (1 + 0.01 * np.arange(20))
              if min(np.abs(v * s - np.round(v * s)).min() for v in w) > 2e-5)
    outs = [orc.inference(x, None, 0.0, ls) for x in ids]
    batch, lens = pad_batch(ids)
    m.length_scale, m.noise_scale = float(ls), 0.0
    Ty = max(o[4] for o in outs)
    y, _, _, _, attn, _, _ = m.inference(torch.from_numpy(batch).cuda(), lens,
                                         noise=torch.zeros(len(ids), 80, Ty).cuda())
    y, attn = y.cpu().numpy(), attn.cpu().numpy()
    worst = 0.0
    for i, (yr, _, ar, _, ty) in enumerate(outs):
        assert int(m.last_y_lengths[i]) == ty, i
        assert np.array_equal(attn[i, :ty, :len(ids[i])], ar), i
        err = float(np.abs(y[i, :, :yr.shape[1]] - yr).max())
        worst = max(worst, err)
        assert err <= 1e-4, (i, err)
    print(f"32 utterances, {int(m.last_y_lengths.sum())} frames, length_scale {ls:.4f}, worst mel error {worst:.2e}")


def test_pwgan_lj_batch_full_size_batched_equals_single():
    """ParallelWaveGAN at tools/pwgan_bench.py's size (32 LJ-profile mel lengths, 4.9 M samples in
    one call, explicit noise): the shortest, median and longest rows of the batched call are
    bit-identical to B = 1 calls on the same mel and noise, and zero past their length. (The oracle
    runs ~2.6 k samples/s, too slow at this size; parity vs the oracle is the small-size tests.)"""
    from tts_amd import ParallelWaveganGenerator
    from tts_amd.spec import PwganConfig, pwgan_spec
    from tts_amd.workload import lj_profile
    _dev()
    sd = synth_state_dict(pwgan_spec(PwganConfig()), 5)
    g = ParallelWaveganGenerator(inference_padding=0)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    g = g.cuda().eval()
    _, M = lj_profile()
    rs = np.random.RandomState(8)
    mel = np.zeros((len(M), 80, max(M)), np.float32)
    for i, m in enumerate(M):
        mel[i, :, :m] = rs.normal(0, 1, (80, m))
    noise = torch.randn(len(M), 1, max(M) * 256, generator=torch.Generator().manual_seed(2)).cuda()
    melt = torch.from_numpy(mel).cuda()
    with torch.no_grad():
        yb = g.inference(melt, lengths=list(M), noise=noise).cpu().numpy()
        for i in (int(np.argmin(M)), len(M) // 2, int(np.argmax(M))):
            n = M[i] * 256
            y1 = g.inference(melt[i:i + 1, :, :M[i]], noise=noise[i:i + 1, :, :n].contiguous()).cpu().numpy()
            assert y1.shape[-1] == n
            assert np.array_equal(yb[i, 0, :n], y1[0, 0]), i
            assert not yb[i, 0, n:].any(), i


def test_c5_chained_shard_vs_oracle_chain():
    """Config C5's per-GPU shard as ONE chained GPU run (tools/c5_bench.py's models and workload):
    GE2E SpeakerEncoder.inference on 16 reference mels (160 frames x 40) -> their 256-d embeddings into
    the multi-speaker Tacotron2 (speaker_embeddings, models/tacotron2.py:152-155) on 16 LJ-profile
    sentences (forced lengths, r = 2) -> the full-band MelGAN (base 512, 8x8x2x2, 3 residual blocks) on
    the batched mels. Every row against the B = 1 oracle chain (Ge2eOracle -> TacoOracle(speaker=...)
    -> MelganOracle.generator): embeddings <= 1e-5, mel <= 1e-4, alignment argmax identical, waveform
    <= 1e-4 and zero past its length (speaker_encoder/model.py:62-88, melgan_generator.py:83-89)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import c5_bench
    from oracle.ge2e_np import Ge2eOracle
    from oracle.taco_np import TacoOracle
    from tts_amd.spec import Ge2eConfig, MelganConfig, TacotronConfig, ge2e_spec, melgan_spec, tacotron2_spec
    from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids
    dev = _dev()
    r, B = 2, 16
    taco, spk, voc = c5_bench.build(dev, r)
    T, M = lj_profile()
    T, M = T[:B], M[:B]
    ids = synthetic_ids(T)
    batch, lens = pad_batch(ids)
    steps = forced_steps(M, r)
    ref_mels = np.random.RandomState(5).normal(0, 1, (B, 160, 40)).astype(np.float32)
    with torch.no_grad():
        emb = spk.inference(torch.from_numpy(ref_mels).to(dev))
        _, post, align, _ = taco.inference(torch.from_numpy(batch).to(dev), text_lengths=lens, max_decoder_steps=steps,
                                           speaker_embeddings=emb)
        assert list(taco.last_steps) == list(steps)
        wav = voc.inference(post.transpose(1, 2), lengths=taco.last_mel_lengths).cpu().numpy()
    emb, post, align = emb.cpu().numpy(), post.cpu().numpy(), align.cpu().numpy()
    tcfg = TacotronConfig(num_speakers=8, speaker_embedding_dim=256)
    tsd = synth_state_dict(tacotron2_spec(tcfg), 11)
    tsd["decoder.stopnet.1.linear_layer.bias"] = np.array([-1e4], np.float32)
    go = Ge2eOracle(synth_state_dict(ge2e_spec(Ge2eConfig()), 12))
    to = TacoOracle(tsd, tcfg.attn_norm, tcfg.r)
    vcfg = MelganConfig(out_channels=1, base_channels=512, upsample_factors=(8, 8, 2, 2), num_res_blocks=3, pqmf=False)
    vo = melgan_oracle(vcfg, synth_state_dict(melgan_spec(vcfg, weight_norm=True), 13))
    worst = [0.0, 0.0, 0.0]
    for i in range(B):
        e = go.inference(ref_mels[i])
        worst[0] = max(worst[0], float(np.abs(emb[i] - e).max()))
        assert worst[0] <= 1e-5, i
        _, p, a, _ = to.inference(ids[i], r, steps[i], speaker=e)
        n = steps[i] * r
        worst[1] = max(worst[1], float(np.abs(post[i, :n] - p).max()))
        assert worst[1] <= MEL_TOL, i
        assert (align[i, :steps[i], :len(ids[i])].argmax(1) == a.argmax(1)).all(), i
        w = vo.generator(p.T)[0]
        assert w.size == 256 * n
        worst[2] = max(worst[2], float(np.abs(wav[i, 0, :w.size] - w).max()))
        assert worst[2] <= WAV_TOL, i
        assert not wav[i, 0, w.size:].any(), i
    print(f"C5 shard, 16 rows: worst embedding {worst[0]:.2e}, mel {worst[1]:.2e}, waveform {worst[2]:.2e}")


def test_c4_glow_pwgan_batch64_vs_oracle():
    """Config C4 at its stated batch of 64 (1 x MI355X): Glow-TTS on 64 LJ-length utterances (the
    LJ profile twice, ids continuing the RandomState(0) stream) with explicit prior noise at
    noise_scale 0.66, every utterance against the oracle at B = 1 (glow_tts.py:159-193: y_lengths and
    the monotonic path exact, mel <= 1e-4); then ParallelWaveGAN on the 64 Glow mels in ONE batched
    call (per-row lengths, inference_padding 0, explicit noise), EVERY row against the fp32 PyTorch
    reference of the generator on the same mel and noise (parallel_wavegan_generator.py:90-125,
    <= 1e-4; the longest rows reach the persistent residual-block kernel's last tiles), and every row
    zero past its length. length_scale avoids ceil ties as in the 32-row test."""
    import dataclasses
    from oracle.glow_np import GlowOracle
    from oracle.pwgan_np import PwganOracle
    from oracle.torch_cpu import PwganTorchCPU
    from tts_amd import GlowTts, ParallelWaveganGenerator
    from tts_amd.spec import GlowConfig, PwganConfig, glow_spec, pwgan_spec
    from tts_amd.workload import lj_profile, pad_batch, synthetic_ids
    _dev()
    B = 64
    cfg = GlowConfig()
    sd = synth_state_dict(glow_spec(cfg), 3)
    m = GlowTts(num_chars=cfg.num_chars)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    T, M = lj_profile()
    T, M = T * 2, M * 2
    ids = synthetic_ids(T)
    orc = GlowOracle(sd)
    w = [np.exp(orc.encode(x)[1].astype(np.float64)).reshape(-1) - 1 for x in ids]
    base = sum(M) / float(sum(np.ceil(np.maximum(v, 0)).sum() for v in w))
    ls = next(s for s in base * (1 + 0.01 * np.arange(40))
              if min(np.abs(v * s - np.round(v * s)).min() for v in w) > 2e-5)
    tys = [int(max(1, np.ceil(np.maximum(v * ls, 0)).sum())) for v in w]
    noise = np.random.RandomState(64).normal(0, 1, (B, 80, max(tys))).astype(np.float32)
    outs = [orc.inference(x, noise[i], 0.66, ls) for i, x in enumerate(ids)]
    batch, lens = pad_batch(ids)
    m.length_scale, m.noise_scale = float(ls), 0.66
    y, _, _, _, attn, _, _ = m.inference(torch.from_numpy(batch).cuda(), lens, noise=torch.from_numpy(noise).cuda())
    yn, attn = y.cpu().numpy(), attn.cpu().numpy()
    worst = 0.0
    for i, (yr, _, ar, _, ty) in enumerate(outs):
        assert int(m.last_y_lengths[i]) == ty, i
        assert np.array_equal(attn[i, :ty, :len(ids[i])], ar), i
        err = float(np.abs(yn[i, :, :yr.shape[1]] - yr).max())
        worst = max(worst, err)
        assert err <= 1e-4, (i, err)
    # ParallelWaveGAN on the batch of 64 Glow mels (each row's own 2 * floor(Ty / 2) frames)
    pcfg = dataclasses.replace(PwganConfig(), inference_padding=0)
    psd = synth_state_dict(pwgan_spec(pcfg), 5)
    g = ParallelWaveganGenerator(inference_padding=0)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in psd.items()})
    g = g.cuda().eval()
    mlens = [o[0].shape[1] for o in outs]
    pnoise = torch.randn(B, 1, max(mlens) * 256, generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        wav = g.inference(y, lengths=mlens, noise=pnoise.cuda()).cpu().numpy()
    # every row against the fp32 PyTorch reference of the generator (oracle/torch_cpu.py
    # PwganTorchCPU, pinned to the reference fixtures on the CPU by test_oracle_golden), run here
    # with PyTorch's own ROCm kernels so that all 64 rows (9 M samples) take seconds; the shortest
    # row also against the numpy oracle and the same PyTorch reference on the CPU
    order = np.argsort(mlens, kind="stable")
    rows_mel = [yn[i, :, :mlens[i]] for i in range(B)]
    rows_noise = [pnoise[i, 0, :mlens[i] * 256].numpy() for i in range(B)]
    refs = PwganTorchCPU(psd, pcfg, device="cuda").inference_batch(rows_mel, rows_noise)
    torch.cuda.synchronize()
    i0 = int(order[0])
    ref_np = PwganOracle(psd, pcfg).inference(rows_mel[i0], rows_noise[i0])
    ref_cpu = PwganTorchCPU(psd, pcfg).inference(rows_mel[i0], rows_noise[i0])
    assert np.abs(refs[i0] - ref_np).max() <= 2e-6 and np.abs(refs[i0] - ref_cpu).max() <= 2e-6
    # the longest row (the persistent kernel's last tiles) against the same reference on the CPU
    i1 = int(order[-1])
    ref_cpu1 = PwganTorchCPU(psd, pcfg).inference(rows_mel[i1], rows_noise[i1])
    assert np.abs(refs[i1] - ref_cpu1).max() <= 2e-6
    assert np.abs(wav[i1, 0, :mlens[i1] * 256] - ref_cpu1).max() <= WAV_TOL
    worst_w, wrow = 0.0, -1
    for i in range(B):
        n = mlens[i] * 256
        werr = float(np.abs(wav[i, 0, :n] - refs[i]).max())
        if werr > worst_w:
            worst_w, wrow = werr, i
        assert werr <= WAV_TOL, (i, werr)
        assert not wav[i, 0, n:].any(), i
    print(f"C4 batch 64: {sum(o[4] for o in outs)} frames, worst mel error {worst:.2e}; PWGAN all 64 rows "
          f"{worst_w:.2e} (row {wrow}, {mlens[wrow]} frames; longest {max(mlens)})")


@pytest.mark.parametrize("B", [64, 48])
def test_tacotron2_persistent_64_row_batch_vs_oracle(B):
    """Batches of 33-64 rows run on the persistent decoder (batch tiles of 64 / 48 rows, then 32 and
    16 as rows finish: launches with MT = 4 or 3, 2, 1) instead of the step graphs: every row against
    its B = 1 oracle run, ragged lengths and forced step counts with the long rows scattered."""
    from oracle.taco_np import TacoOracle
    from tts_amd._lib import get_engine
    from tts_amd.spec import TacotronConfig
    _dev()
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=29, overrides={}, stop_bias=-1e4, cfg=cfg)
    m = build_taco(cfg, sd)
    r = 2
    m.decoder.set_r(r)
    rs = np.random.RandomState(B)
    lens = [int(x) for x in rs.randint(1, 60, B)]
    steps = [int(x) for x in rs.randint(2, 12, B)]
    for i in range(5, B, 11):
        steps[i] = 30 + i % 7
    batch = np.zeros((B, max(lens)), np.int64)
    for i, L in enumerate(lens):
        batch[i, :L] = rs.randint(1, 129, L)
    dec, post, align, stop = m.inference(torch.from_numpy(batch).cuda(), text_lengths=lens, max_decoder_steps=steps)
    assert list(m.last_steps) == steps
    path, launches = get_engine("cuda:0").decoder_stats()
    assert path == 1 and len(launches) == (B + 15) // 16, launches
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    dec, post, align = dec.cpu().numpy(), post.cpu().numpy(), align.cpu().numpy()
    for i, L in enumerate(lens):
        d, p, a, _ = orc.inference(batch[i, :L], r, steps[i])
        n = steps[i] * r
        assert np.abs(dec[i, :n] - d).max() <= MEL_TOL, i
        assert np.abs(post[i, :n] - p).max() <= MEL_TOL, i
        assert np.abs(align[i, :steps[i], :L] - a).max() <= 1e-5, i
        assert not post[i, n:].any()


def test_tacotron2_multispeaker_40_rows_vs_oracle():
    """Multi-speaker decoding (external 256-d embeddings, models/tacotron2.py:152-155) above the
    former 32-row cap: 40 rows in one call (batch tiles 48 -> 32 -> 16), each row against the oracle
    with its own speaker vector."""
    from oracle.taco_np import TacoOracle
    from tts_amd.spec import TacotronConfig
    _dev()
    cfg = TacotronConfig(num_speakers=2, speaker_embedding_dim=256)
    _, sd = taco_state_dict(None, seed=31, overrides={}, stop_bias=-1e4, cfg=cfg)
    m = build_taco(cfg, sd)
    r = 2
    m.decoder.set_r(r)
    B = 40
    rs = np.random.RandomState(40)
    lens = [int(x) for x in rs.randint(3, 40, B)]
    steps = [int(x) for x in rs.randint(3, 20, B)]
    emb = rs.randn(B, 256).astype(np.float32)
    emb /= np.linalg.norm(emb, axis=1, keepdims=True)
    batch = np.zeros((B, max(lens)), np.int64)
    for i, L in enumerate(lens):
        batch[i, :L] = rs.randint(1, 129, L)
    _, post, _, _ = m.inference(torch.from_numpy(batch).cuda(), text_lengths=lens, max_decoder_steps=steps,
                                speaker_embeddings=torch.from_numpy(emb).cuda())
    assert list(m.last_steps) == steps
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    post = post.cpu().numpy()
    for i, L in enumerate(lens):
        _, p, _, _ = orc.inference(batch[i, :L], r, steps[i], speaker=emb[i])
        assert np.abs(post[i, :steps[i] * r] - p).max() <= MEL_TOL, i


@pytest.mark.parametrize("r,n", [(2, 1), (2, 7), (1, 4)])
def test_tacotron2_decoder_state_matches_reference(r, n):
    """Per-stage decoder parity through tts_taco_decoder_state: after exactly n decoder steps (both
    fixture utterances in one batched call, forced to n steps), the attention_rnn and decoder_rnn
    LSTM states, the context and the attention weights / cumulative weights equal the state the
    reference leaves on `self` (layers/tacotron2.py:217-233,259-298; common_layers.py:251-260)."""
    _dev()
    fx = load_fixture("taco_state")
    cfg, sd = taco_state_dict(fx, stop_bias=-1e4)
    m = build_taco(cfg, sd)
    m.decoder.set_r(r)
    ids = [fx[f"r{r}_n{n}_u{u}_ids"] for u in range(2)]
    batch = np.zeros((2, max(len(x) for x in ids)), np.int64)
    for i, x in enumerate(ids):
        batch[i, :len(x)] = x
    m.inference(torch.from_numpy(batch).cuda(), text_lengths=[len(x) for x in ids], max_decoder_steps=n)
    assert list(m.last_steps) == [n, n]
    st = {k: v.cpu().numpy() for k, v in m.decoder_state().items()}
    for u in range(2):
        k = f"r{r}_n{n}_u{u}"
        L = len(ids[u])
        for a in ("query", "attention_rnn_cell_state", "decoder_hidden", "decoder_cell", "context"):
            assert np.abs(st[a][u] - fx[f"{k}_{a}"]).max() <= 1e-5, (k, a)
        for a in ("attention_weights", "attention_weights_cum"):
            assert np.abs(st[a][u, :L] - fx[f"{k}_{a}"]).max() <= 1e-5, (k, a)
            assert not st[a][u, L:].any(), (k, a)
