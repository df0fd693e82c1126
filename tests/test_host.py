"""CPU: host-side logic of the drop-in boundary (no GPU, no library compute calls)."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from helpers import GOLDEN
from tts_amd import (MultibandMelganGenerator, Tacotron2, load_config, setup_generator,  # noqa: F401
                     setup_model)
from tts_amd.spec import MelganConfig, TacotronConfig, tacotron2_spec
from tts_amd.weights import splitmix64_uniform, synth_state_dict
from tts_amd.workload import forced_steps, lj_profile, lpt_shards, pad_batch, replicated_workload, synthetic_ids


def _keys(sd):
    return {k: (tuple(v.shape), str(v.dtype).replace("torch.", "")) for k, v in sd.items()}


def _ref_keys(name):
    d = json.load(open(os.path.join(GOLDEN, "state_dict_keys.json")))
    return {k: (tuple(s), t) for k, s, t in d[name]}


def test_tacotron2_state_dict_keys_match_reference_checkpoint():
    m = Tacotron2(num_chars=129, num_speakers=0, r=7, attn_norm="sigmoid", double_decoder_consistency=True, ddc_r=7)
    assert _keys(m.state_dict()) == _ref_keys("tacotron2_ddc")


def test_mbmelgan_state_dict_keys_match_reference_checkpoint():
    v = MultibandMelganGenerator(upsample_factors=(8, 4, 2), num_res_blocks=4)
    assert _keys(v.state_dict()) == _ref_keys("multiband_melgan")
    v.remove_weight_norm()
    assert _keys(v.state_dict()) == _ref_keys("multiband_melgan_wn_removed")


def test_remove_weight_norm_matches_definition():
    cfg = MelganConfig()
    v = MultibandMelganGenerator(upsample_factors=cfg.upsample_factors, num_res_blocks=cfg.num_res_blocks)
    from helpers import melgan_state_dict
    _, sd = melgan_state_dict(7)
    full = v.state_dict()
    for k, t in sd.items():
        full[k] = torch.from_numpy(t)
    v.load_state_dict(full)
    g, vv = sd["layers.3.weight_g"], sd["layers.3.weight_v"]
    v.remove_weight_norm()
    w = v.state_dict()["layers.3.weight"].numpy()
    ref = vv / np.sqrt((vv.astype(np.float64) ** 2).sum(axis=(1, 2), keepdims=True)) * g
    assert np.abs(w - ref).max() <= 1e-6


def test_synthetic_weights_are_version_stable():
    u = splitmix64_uniform(12345, 8)
    assert np.all((u >= -1) & (u < 1))
    sd = synth_state_dict(tacotron2_spec(TacotronConfig()), 0)
    h = hashlib.sha256(sd["decoder.decoder_rnn.weight_hh"].tobytes()).hexdigest()
    again = synth_state_dict(tacotron2_spec(TacotronConfig()), 0)["decoder.decoder_rnn.weight_hh"]
    assert hashlib.sha256(again.tobytes()).hexdigest() == h
    assert sd["decoder.decoder_rnn.weight_hh"].dtype == np.float32


def test_multispeaker_state_dict_keys_and_shapes():
    """models/tacotron2.py:50-58: a learned (num_speakers, 512) table, decoder_in_features 1024;
    per-sample embeddings (tacotron_abstract.py:76-81): no table, 512 + speaker_embedding_dim."""
    m = Tacotron2(num_chars=129, num_speakers=4, double_decoder_consistency=True, ddc_r=7)
    sd = m.state_dict()
    assert tuple(sd["speaker_embedding.weight"].shape) == (4, 512)
    assert tuple(sd["decoder.attention.inputs_layer.linear_layer.weight"].shape) == (128, 1024)
    assert tuple(sd["decoder.linear_projection.linear_layer.weight"].shape) == (560, 2048)
    assert tuple(sd["coarse_decoder.decoder_rnn.weight_ih"].shape) == (4096, 2048)
    m2 = Tacotron2(num_chars=129, num_speakers=2, speaker_embedding_dim=256)
    sd2 = m2.state_dict()
    assert "speaker_embedding.weight" not in sd2
    assert tuple(sd2["decoder.attention_rnn.weight_ih"].shape) == (4096, 256 + 768)


# (Graves attention with speaker embeddings is supported since round 3: test_gpu_parity graves_spk)
@pytest.mark.parametrize("kw", [dict(gst=True), dict(trans_agent=True), dict(prenet_type="xyz"),
                                dict(location_attn=False)])
def test_unsupported_tacotron_variants_raise(kw):
    with pytest.raises(NotImplementedError):
        Tacotron2(num_chars=129, **kw)


def test_unknown_attention_norm_raises_valueerror():
    with pytest.raises(ValueError):
        Tacotron2(num_chars=129, attn_norm="entmax")


def test_no_cpu_fallback():
    m = Tacotron2(num_chars=129, r=2, attn_norm="sigmoid")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m.inference(torch.ones(1, 5, dtype=torch.long))
    v = MultibandMelganGenerator(upsample_factors=(8, 4, 2), num_res_blocks=4)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        v.inference(torch.zeros(1, 80, 8))


def test_decoder_knobs():
    m = Tacotron2(num_chars=129, r=7, attn_norm="sigmoid")
    assert m.decoder.max_decoder_steps == 1000 and m.decoder.r == 7 and m.decoder.stop_threshold == 0.5
    m.decoder.set_r(2)
    m.decoder.max_decoder_steps = 3000
    assert m.decoder.r == 2 and m.decoder.r_init == 7


CONFIG_TTS = """{
  // Tacotron2-DDC style config (comments are stripped like TTS/utils/io.py:20-34)
  "model": "Tacotron2",
  "r": 7,
  "audio": {"num_mels": 80, "fft_size": 1024, "sample_rate": 22050},
  "use_gst": false,
  "gst": {"gst_embedding_dim": 512, "gst_num_heads": 4, "gst_style_tokens": 10, "gst_use_speaker_embedding": false},
  "attention_type": "original", "attention_heads": 4, "attention_norm": "sigmoid", "windowing": false,
  "prenet_type": "original", "prenet_dropout": false, "use_forward_attn": false, "transition_agent": false,
  "forward_attn_mask": false, "location_attn": true, "separate_stopnet": true,
  "bidirectional_decoder": false, "double_decoder_consistency": true, "ddc_r": 7
}
"""

CONFIG_VOC = """{
  "audio": {"num_mels": 80},
  "generator_model": "multiband_melgan_generator",  // MB-MelGAN
  "generator_model_params": {"upsample_factors": [8, 4, 2], "num_res_blocks": 4}
}
"""


def test_factories_build_drop_in_models(tmp_path):
    p = tmp_path / "config.json"
    p.write_text(CONFIG_TTS)
    c = load_config(str(p))
    assert c.model == "Tacotron2" and c.attention_norm == "sigmoid"
    m = setup_model(129, 0, c)
    assert isinstance(m, Tacotron2) and m.decoder.r_init == 7 and m.attn_norm == "sigmoid"
    assert _keys(m.state_dict()) == _ref_keys("tacotron2_ddc")
    q = tmp_path / "vocoder.json"
    q.write_text(CONFIG_VOC)
    v = setup_generator(load_config(str(q)))
    assert isinstance(v, MultibandMelganGenerator) and v.hop == 256
    assert _keys(v.state_dict()) == _ref_keys("multiband_melgan")


def test_lj_profile_and_workload():
    T, M = lj_profile()
    assert len(T) == 32 and sum(T) == 3346 and sum(M) == 19112 and max(T) == 168 and max(M) == 857
    steps = forced_steps(M, 2)
    assert all(s * 2 >= m > (s - 1) * 2 for s, m in zip(steps, M))
    ids = synthetic_ids(T)
    assert [len(x) for x in ids] == T and min(x.min() for x in ids) >= 1 and max(x.max() for x in ids) <= 128
    batch, lens = pad_batch(ids[:3])
    assert batch.shape == (3, max(T[:3])) and list(lens) == T[:3]
    assert (batch[0, lens[0]:] == 0).all()


def test_lpt_shards_partition_and_balance():
    T, M = lj_profile()
    costs = forced_steps(M, 2)
    for n in (1, 2, 4, 8):
        sh = lpt_shards(costs, n)
        flat = sorted(i for s in sh for i in s)
        assert flat == list(range(len(costs)))
        assert max(len(s) for s in sh) - min(len(s) for s in sh) <= 1
        loads = [sum(costs[i] for i in s) for s in sh]
        assert max(loads) - min(loads) <= max(costs)


def test_replicated_workload_weak_scaling():
    for n in (1, 2, 4, 8):
        T, M, shards = replicated_workload(n, 32)
        assert len(shards) == n and all(len(s) == 32 for s in shards)
        assert sorted(i for s in shards for i in s) == list(range(32 * n))
        assert sum(M[i] for i in shards[-1]) == 19112
        # bench.py's plan (tts_amd.multigpu.shard_plan, LPT on the step counts) gives every rank one
        # copy of each profile utterance: the per-rank work of C2
        from tts_amd.multigpu import shard_plan
        plan = shard_plan([s_ * 1e6 + t_ for s_, t_ in zip(forced_steps(M, 2), T)], n)
        assert all(sorted(i % 32 for i in s) == list(range(32)) for s in plan)


def test_glow_tts_constructor_and_keys():
    """glow_tts.py:17-95 with the gated-conv encoder: checkpoint key layout; other encoders raise."""
    from tts_amd import GlowTts
    m = GlowTts(num_chars=130)
    sd = m.state_dict()
    assert tuple(sd["encoder.emb.weight"].shape) == (130, 192)
    assert tuple(sd["encoder.proj_m.weight"].shape) == (80, 192, 1)
    assert tuple(sd["decoder.flows.1.weight"].shape) == (4, 4)
    assert m.noise_scale == 0.66 and m.length_scale == 1.
    for kw in (dict(encoder_type="transformer", rel_attn_window_size=4, use_encoder_prenet=True),
               dict(encoder_type="transformer"), dict(mean_only=False)):
        with pytest.raises(NotImplementedError):
            GlowTts(num_chars=130, **kw)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m.inference(torch.ones(1, 5, dtype=torch.long), [5])


def test_glow_tts_multispeaker_keys_and_misuse():
    """Multi-speaker GlowTts (glow_tts.py:97-99, encoder.py:112-114, glow.py:87-91): emb_g, the
    duration predictor's hidden + c_in inputs, one weight-normed cond_layer per coupling block, in
    the reference's key order (pinned against the reference module by make_golden.py glow_spk); g
    misuse fails before any GPU work, with the reference's exception types."""
    from tts_amd import GlowTts
    m = GlowTts(num_chars=130, num_speakers=4, c_in_channels=36)
    sd = m.state_dict()
    keys = list(sd)
    assert keys[-1] == "emb_g.weight" and tuple(sd["emb_g.weight"].shape) == (4, 36)
    assert tuple(sd["encoder.duration_predictor.conv_1.weight"].shape) == (256, 192 + 36, 3)
    assert tuple(sd["decoder.flows.2.wn.cond_layer.weight_v"].shape) == (2 * 192 * 4, 36, 1)
    assert keys.index("decoder.flows.2.wn.cond_layer.bias") == keys.index("decoder.flows.2.wn.res_skip_layers.3.weight_v") + 1
    assert sum(k.endswith("cond_layer.weight_g") for k in keys) == 12
    x = torch.ones(1, 5, dtype=torch.long)
    with pytest.raises(RuntimeError, match="pass g"):
        m.inference(x, [5])
    with pytest.raises(IndexError):
        m.inference(x, [5], g=torch.tensor([4]))
    with pytest.raises(AttributeError, match="emb_g"):
        GlowTts(num_chars=130).inference(x, [5], g=torch.tensor([0]))
    # setup_model's multi-speaker call (num_speakers > 1, c_in_channels = 0): an empty emb_g, and g
    # cannot reach a cond_layer
    m0 = GlowTts(num_chars=130, num_speakers=4)
    assert tuple(m0.state_dict()["emb_g.weight"].shape) == (4, 0)
    with pytest.raises(AttributeError, match="cond_layer"):
        m0.inference(x, [5], g=torch.tensor([0]))


def test_pwgan_keys_match_reference_and_factory():
    """parallel_wavegan_generator.py:16-88 checkpoint keys (pinned against the reference module by
    make_golden.py pwgan), remove_weight_norm folding, setup_generator dispatch."""
    from tts_amd import ParallelWaveganGenerator
    from tts_amd.spec import PwganConfig, pwgan_spec
    g = ParallelWaveganGenerator()
    assert [(k, tuple(v.shape)) for k, v in g.state_dict().items()] == \
        [(n, tuple(s)) for n, s, _ in pwgan_spec(PwganConfig())]
    assert tuple(g.state_dict()["upsample_net.upsample.up_layers.7.weight_v"].shape) == (1, 1, 1, 9)
    g.remove_weight_norm()
    sd = g.state_dict()
    assert "conv_layers.29.conv.weight" in sd and "conv_layers.29.conv.weight_g" not in sd
    c = {"generator_model": "parallel_wavegan_generator", "audio": {"num_mels": 80},
         "generator_model_params": {"upsample_factors": [4, 4, 4, 4], "stacks": 3, "num_res_blocks": 30}}
    v = setup_generator(c)
    assert isinstance(v, ParallelWaveganGenerator) and v.hop == 256
    with pytest.raises(NotImplementedError):
        ParallelWaveganGenerator(res_channels=32)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        v.inference(torch.zeros(1, 80, 4))


def test_bidirectional_decoder_keys():
    """bidirectional_decoder=True: decoder_backward.* mirrors decoder.* (tacotron_abstract.py:104-105),
    registered before coarse_decoder (checked against the reference module when it was built)."""
    m = Tacotron2(num_chars=129, r=7, double_decoder_consistency=True, ddc_r=7, bidirectional_decoder=True)
    keys = list(m.state_dict().keys())
    dec = [k for k in keys if k.startswith("decoder.")]
    bwd = [k for k in keys if k.startswith("decoder_backward.")]
    assert bwd == ["decoder_backward." + k[len("decoder."):] for k in dec]
    assert keys.index(bwd[-1]) < keys.index("coarse_decoder.prenet.linear_layers.0.linear_layer.weight")


class _FakeTacoEngine:
    """Stands in for the library context: records the chunks the host logic hands it and fills
    each row's outputs with recognisable values up to that row's own step count."""

    def __init__(self):
        import threading
        self.lock = threading.RLock()
        self.taco_key = None
        self.calls = []

    def load_tacotron(self, *a, **k):
        pass

    def taco_infer(self, ids, lens, r, ms, S_cap, thr, dec, post, align, stop, speaker_ids=None,
                   speaker_embeddings=None):
        assert self.lock._is_owned()  # the model holds the engine lock across the call
        nb = ids.shape[0]
        self.calls.append((nb, S_cap, ids.shape[1]))
        steps = np.asarray(ms, np.int32).copy()
        dec.zero_(), post.zero_(), align.zero_(), stop.zero_()
        for i in range(nb):
            tag = float(ids[i, 0])
            dec[i, :steps[i] * r] = tag
            post[i, :steps[i] * r] = tag + 0.5
            align[i, :steps[i], :int(lens[i])] = tag
            stop[i, :steps[i]] = tag
        return steps, np.full(nb, 2, np.int32)


def test_tacotron2_multichunk_join_ragged_steps(monkeypatch):
    """B = 70 splits into chunks of 64 and 6 that decode to different S_cap (the second chunk
    longer than the first, then shorter): every row keeps its own frames and zero padding, in
    the caller's order (the join used to assume equal chunk lengths)."""
    import tts_amd.tacotron2 as tmod
    eng = _FakeTacoEngine()
    monkeypatch.setattr(tmod, "get_engine", lambda dev: eng)
    m = Tacotron2(num_chars=129, r=7, attn_norm="sigmoid")
    m.decoder.set_r(2)
    m.decoder.verbose = False
    B = 70
    rs = np.random.RandomState(0)
    for long_chunk in (0, 1):
        lens = rs.randint(1, 30, B)
        steps = rs.randint(1, 6, B)
        steps[64 + 2 if long_chunk else 5] = 17  # the longest row sits in one chunk only
        ids = np.zeros((B, lens.max()), np.int64)
        for i in range(B):
            ids[i, :lens[i]] = i + 1
        eng.calls.clear()
        dec, post, align, stop = m.inference(torch.from_numpy(ids), text_lengths=lens, max_decoder_steps=steps)
        assert [c[0] for c in eng.calls] == [64, 6]
        S = int(steps.max())
        assert dec.shape == (B, 2 * S, 80) and post.shape == (B, 2 * S, 80)
        assert align.shape == (B, S, lens.max()) and stop.shape == (B, S, 1)
        for i in range(B):
            M = 2 * steps[i]
            assert (dec[i, :M] == i + 1).all() and not dec[i, M:].any()
            assert (post[i, :M] == i + 1.5).all() and not post[i, M:].any()
            assert (align[i, :steps[i], :lens[i]] == i + 1).all() and not align[i, :, lens[i]:].any()
            assert not align[i, steps[i]:].any() and not stop[i, steps[i]:].any()
        assert list(m.last_steps) == list(steps)


def test_single_speaker_model_ignores_speaker_arguments(monkeypatch):
    """models/tacotron2.py:152: speaker_ids / speaker_embeddings are ignored when num_speakers <= 1."""
    import tts_amd.tacotron2 as tmod
    eng = _FakeTacoEngine()
    monkeypatch.setattr(tmod, "get_engine", lambda dev: eng)
    m = Tacotron2(num_chars=129, r=2, attn_norm="sigmoid")
    m.decoder.verbose = False
    ids = torch.ones(1, 5, dtype=torch.long)
    a = m.inference(ids, max_decoder_steps=3)
    b = m.inference(ids, speaker_ids=torch.tensor([3]), speaker_embeddings=torch.ones(1, 256),
                    max_decoder_steps=3)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
