"""Shared fixture plumbing for the parity tests (weights are regenerated from seeds)."""
import json
import os

import numpy as np
import torch

from tts_amd.spec import MelganConfig, TacotronConfig, melgan_layers, melgan_spec, tacotron2_spec
from tts_amd.weights import synth_state_dict

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixture(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def taco_cfg(fx):
    return TacotronConfig(**json.loads(str(fx["cfg"])))


def taco_state_dict(fx, r=None, seed=None, overrides=None, stop_bias=None, cfg=None):
    cfg = cfg or taco_cfg(fx)
    if seed is None:  # per-r seed when the fixture's stop-margin search moved it between r values
        seed = int(fx[f"r{r}_seed"]) if r is not None and f"r{r}_seed" in fx.files else int(fx["seed"])
    ov = json.loads(str(fx["overrides"])) if overrides is None else overrides
    sd = synth_state_dict(tacotron2_spec(cfg), seed, ov)
    if stop_bias is None and r is not None:
        stop_bias = float(fx[f"r{r}_stop_bias"])
    if stop_bias is not None:
        sd["decoder.stopnet.1.linear_layer.bias"] = np.array([stop_bias], np.float32)
    return cfg, sd


def build_taco(cfg, sd, device="cuda"):
    from tts_amd import Tacotron2
    m = Tacotron2(num_chars=cfg.num_chars, num_speakers=cfg.num_speakers, r=cfg.r, attn_norm=cfg.attn_norm,
                  double_decoder_consistency=cfg.double_decoder_consistency, ddc_r=cfg.ddc_r,
                  speaker_embedding_dim=cfg.speaker_embedding_dim, prenet_type=cfg.prenet_type,
                  attn_win=cfg.windowing, forward_attn=cfg.forward_attn, trans_agent=cfg.trans_agent,
                  forward_attn_mask=cfg.forward_attn_mask, attn_type=cfg.attn_type, attn_K=cfg.attn_K,
                  bidirectional_decoder=cfg.bidirectional_decoder)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.to(device).eval()


def melgan_state_dict(seed, cfg=None):
    cfg = cfg or MelganConfig()
    return cfg, synth_state_dict(melgan_spec(cfg, weight_norm=True), seed)


def build_melgan(cfg, sd, device="cuda"):
    from tts_amd import MultibandMelganGenerator
    v = MultibandMelganGenerator(in_channels=cfg.in_channels, out_channels=cfg.out_channels,
                                 base_channels=cfg.base_channels, upsample_factors=cfg.upsample_factors,
                                 num_res_blocks=cfg.num_res_blocks)
    full = v.state_dict()
    for k, t in sd.items():
        full[k] = torch.from_numpy(t)
    v.load_state_dict(full)
    v.remove_weight_norm()
    return v.to(device).eval()


def melgan_oracle(cfg, sd):
    from oracle.melgan_np import MelganOracle
    from tts_amd.pqmf import pqmf_filters
    return MelganOracle(sd, melgan_layers(cfg), pqmf_filters()[1])
