"""Config C5 on one GPU: multi-speaker Tacotron2 conditioned on GE2E speaker embeddings + full-band
MelGAN, the per-GPU shard of "batch 128 over 8 MI355X" (16 utterances).

One step = GE2E `SpeakerEncoder.inference` on one reference utterance per sentence (synthetic 40-bin
mels, 160 frames), multi-speaker `Tacotron2.inference` with those 256-d embeddings
(speaker_embedding_dim = 256, `models/tacotron2.py:50-58,152-155`), then `MelganGenerator.inference`
(`melgan_generator.py`, base 512, upsampling 8x8x2x2, 3 residual blocks). Lengths: the first 16
LJ-profile utterances stand in for LibriTTS sentences (no dataset offline); forced decoder lengths
as in bench.py. Random weights (tts_amd.weights). Prints one JSON line. Not part of the library.
  python tools/c5_bench.py [--steps 10 --warmup 2 --batch 16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tts_amd import MelganGenerator, SpeakerEncoder, Tacotron2  # noqa: E402
from tts_amd.spec import (Ge2eConfig, MelganConfig, TacotronConfig, ge2e_spec, melgan_spec,  # noqa: E402
                          tacotron2_spec)
from tts_amd.weights import synth_state_dict  # noqa: E402
from tts_amd.workload import HOP, SAMPLE_RATE, forced_steps, lj_profile, pad_batch, synthetic_ids  # noqa: E402


def build(dev, r):
    tcfg = TacotronConfig(num_speakers=8, speaker_embedding_dim=256)
    tsd = synth_state_dict(tacotron2_spec(tcfg), 11)
    tsd["decoder.stopnet.1.linear_layer.bias"] = np.array([-1e4], np.float32)  # forced length
    taco = Tacotron2(num_chars=tcfg.num_chars, num_speakers=tcfg.num_speakers, r=tcfg.r, attn_norm=tcfg.attn_norm,
                     double_decoder_consistency=True, ddc_r=tcfg.ddc_r, speaker_embedding_dim=256)
    taco.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in tsd.items()})
    taco = taco.to(dev).eval()
    taco.decoder.set_r(r)
    taco.decoder.verbose = False
    gcfg = Ge2eConfig()
    spk = SpeakerEncoder(gcfg.input_dim, gcfg.proj_dim, gcfg.lstm_dim, gcfg.num_lstm_layers,
                         gcfg.use_lstm_with_projection)
    spk.load_state_dict({k: torch.from_numpy(v) for k, v in synth_state_dict(ge2e_spec(gcfg), 12).items()})
    spk = spk.to(dev).eval()
    vcfg = MelganConfig(out_channels=1, base_channels=512, upsample_factors=(8, 8, 2, 2), num_res_blocks=3,
                        pqmf=False)
    voc = MelganGenerator(in_channels=80, out_channels=1, base_channels=512, upsample_factors=(8, 8, 2, 2),
                          num_res_blocks=3)
    full = voc.state_dict()
    for k, v in synth_state_dict(melgan_spec(vcfg, weight_norm=True), 13).items():
        full[k] = torch.from_numpy(v)
    voc.load_state_dict(full)
    voc.remove_weight_norm()
    voc.inference_padding = 0
    return taco, spk, voc.to(dev).eval()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--r", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    taco, spk, voc = build(dev, a.r)
    T, M = lj_profile()
    T, M = T[:a.batch], M[:a.batch]
    batch, lens = pad_batch(synthetic_ids(T))
    ids = torch.from_numpy(batch).to(dev)
    steps = forced_steps(M, a.r)
    ref = torch.from_numpy(np.random.RandomState(5).normal(0, 1, (a.batch, 160, 40)).astype(np.float32)).to(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]

    def one(record=False):
        if record:
            ev[0].record()
        emb = spk.inference(ref)
        if record:
            ev[1].record()
        _, post, _, _ = taco.inference(ids, text_lengths=lens, max_decoder_steps=steps, speaker_embeddings=emb)
        if record:
            ev[2].record()
        wav = voc.inference(post.transpose(1, 2), lengths=taco.last_mel_lengths)
        if record:
            ev[3].record()
        return int(taco.last_mel_lengths.sum()), wav

    for _ in range(a.warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    frames = 0
    for _ in range(a.steps):
        frames += one()[0]
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    per = frames // a.steps
    one(record=True)
    torch.cuda.synchronize()
    split = [ev[i].elapsed_time(ev[i + 1]) for i in range(3)]
    print(json.dumps({
        "metric": "mel-frames/s (C5 per-GPU shard: GE2E + multi-speaker Tacotron2 + MelGAN)",
        "value": round(per / dt, 1), "unit": "mel-frames/s", "ms_per_step": round(dt * 1e3, 3),
        "e2e_rtf": dt / (per * HOP / SAMPLE_RATE), "batch": a.batch, "r": a.r, "frames": per,
        "ge2e_ms": round(split[0], 3), "tacotron2_ms": round(split[1], 3), "melgan_ms": round(split[2], 3),
        "data": "synthetic (LJ-profile lengths stand in for LibriTTS, 160-frame reference mels, random weights)"}))


if __name__ == "__main__":
    main()
