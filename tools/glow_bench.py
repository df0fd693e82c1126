"""Glow-TTS inference throughput on the LJSpeech-shaped batch (32 utterances, lj_profile lengths).

Synthetic weights (tts_amd.weights) and ids; length_scale is calibrated once so the batch produces
the LJ profile's mel frame count (19112 frames for 3346 characters), since random duration
predictor weights give arbitrary durations. Prints one JSON line: mel frames/s and ms per call.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tts_amd import GlowTts  # noqa: E402
from tts_amd.spec import GlowConfig, glow_spec  # noqa: E402
from tts_amd.weights import synth_state_dict  # noqa: E402
from tts_amd.workload import lj_profile, pad_batch, synthetic_ids  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--cpu-utts", type=int, default=0)
    a = ap.parse_args()
    T, M = lj_profile()
    T = [T[i % len(T)] for i in range(a.batch)]  # batch 64 (config C4): the 32-utterance profile twice
    M = [M[i % len(M)] for i in range(a.batch)]
    cfg = GlowConfig()
    m = GlowTts(num_chars=cfg.num_chars)
    sd = synth_state_dict(glow_spec(cfg), 3)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    batch, lens = pad_batch(synthetic_ids(T))
    x = torch.from_numpy(batch).cuda()
    m.inference(x, lens)
    m.length_scale = sum(M) / float(m.last_y_lengths.sum())
    for _ in range(a.warmup):
        m.inference(x, lens)
    frames = int(m.last_y_lengths.sum())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        m.inference(x, lens)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    out = {"metric": "glow_tts_mel_frames_per_sec", "value": frames / dt, "ms_per_call": dt * 1e3,
           "frames": frames, "chars": int(sum(T)), "batch": a.batch, "Ty": int(m.last_y_lengths.max()),
           "length_scale": m.length_scale}
    if a.cpu_utts:  # the numpy oracle (test infrastructure) on the first utterances, B = 1 each
        from oracle.glow_np import GlowOracle
        from threadpoolctl import threadpool_limits
        cores = int(os.environ.get("OMP_NUM_THREADS", "16"))
        orc = GlowOracle(sd)
        ids = synthetic_ids(T)
        n = 0
        with threadpool_limits(cores):
            t0 = time.perf_counter()
            for i in range(a.cpu_utts):
                n += orc.inference(ids[i], None, 0.66, m.length_scale)[4]
            ct = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": n / ct, "unit": "mel-frames/s", "cores": cores, "kind": "port",
                               "sample": f"first {a.cpu_utts} utterances, B=1, numpy fp32 oracle, {ct:.1f} s"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
