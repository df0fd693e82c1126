"""ParallelWaveGAN generator throughput on the LJSpeech-shaped batch: the 32 lj_profile mel lengths
(19112 frames) as one ragged batch, synthetic weights and mels. Prints one JSON line: output samples
per second (real samples, hop * (M + 2 * pad) per row), ms per call and the residual-block kernel's
average duration from HIP events (per layer launch)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tts_amd import ParallelWaveganGenerator  # noqa: E402
from tts_amd.spec import PwganConfig, pwgan_spec  # noqa: E402
from tts_amd.weights import synth_state_dict  # noqa: E402
from tts_amd.workload import lj_profile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--cpu-frames", type=int, default=0)
    ap.add_argument("--dump", default="", help="save the last call's waveforms (.npy) for bit-identity checks")
    a = ap.parse_args()
    _, M = lj_profile()
    M = [M[i % len(M)] for i in range(a.batch)]  # batch 64 (config C4): the 32-utterance profile twice
    g = ParallelWaveganGenerator()
    g.load_state_dict({k: torch.from_numpy(v) for k, v in synth_state_dict(pwgan_spec(PwganConfig()), 5).items()})
    g.remove_weight_norm()
    g = g.cuda().eval()
    rs = np.random.RandomState(0)
    mel = np.zeros((len(M), 80, max(M)), np.float32)
    for i, m in enumerate(M):
        mel[i, :, :m] = rs.uniform(-1, 1, size=(80, m))
    mel = torch.from_numpy(mel).cuda()
    T = 256 * (max(M) + 4)
    torch.manual_seed(0)  # the same prior in every process (--dump comparisons)
    noise = torch.randn(len(M), 1, T, device="cuda")
    for _ in range(a.warmup):
        g.inference(mel, lengths=M, noise=noise)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        y = g.inference(mel, lengths=M, noise=noise)
    torch.cuda.synchronize()
    if a.dump:
        np.save(a.dump, y.cpu().numpy())
    dt = (time.perf_counter() - t0) / a.steps
    samples = 256 * (sum(M) + 4 * len(M))
    flops = samples * 30 * 2 * (128 * 272 + 128 * 64)
    out = {"metric": "pwgan_samples_per_sec", "value": samples / dt, "ms_per_call": dt * 1e3,
           "samples": samples, "mel_frames": int(sum(M)), "batch": len(M),
           "residual_block_tflops_lower_bound": flops / dt / 1e12}
    if a.cpu_frames:  # the numpy oracle (test infrastructure) on a bounded sample, as bench.py does
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
        from oracle.pwgan_np import PwganOracle
        from threadpoolctl import threadpool_limits
        cores = int(os.environ.get("OMP_NUM_THREADS", "16"))
        sd = synth_state_dict(pwgan_spec(PwganConfig()), 5)
        orc = PwganOracle(sd, PwganConfig())
        m0 = np.random.RandomState(1).uniform(-1, 1, size=(80, a.cpu_frames)).astype(np.float32)
        nz = np.random.RandomState(2).randn(256 * (a.cpu_frames + 4)).astype(np.float32)
        with threadpool_limits(cores):
            t0 = time.perf_counter()
            orc.inference(m0, nz)
            ct = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": 256 * (a.cpu_frames + 4) / ct, "unit": "samples/s", "cores": cores,
                               "kind": "port", "sample": f"one {a.cpu_frames}-frame mel, numpy fp32 oracle, {ct:.1f} s"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
