"""Host time inside one bench step (the device-resident C2 step of bench.py): where the host spends
the Tacotron2 -> MB-MelGAN hand-over. Wall-clock stamps around the library calls, cProfile of a
few steps, top functions by own time.

    python tools/host_gap.py
"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    taco, _, voc, _, _, _ = bench.build_models(dev)
    taco.decoder.verbose = False
    T, M = lj_profile()
    ids = synthetic_ids(T)
    batch, lens = pad_batch(ids)
    x = torch.from_numpy(batch).to(dev)
    taco.decoder.set_r(2)
    steps = forced_steps(M, 2)

    def step(stamps=None):
        t0 = time.perf_counter()
        _, post, _, _ = taco.inference(x, text_lengths=lens, max_decoder_steps=steps)
        t1 = time.perf_counter()
        wav = voc.inference(post.transpose(1, 2), lengths=taco.last_mel_lengths)
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if stamps is not None:
            stamps.append((t1 - t0, t2 - t1, t3 - t2))
        return wav

    for _ in range(3):
        step()
    st = []
    for _ in range(10):
        step(st)
    a = np.array(st) * 1e3
    print("per step (ms, median of 10): taco call %.3f  voc call (enqueue) %.3f  voc drain %.3f" %
          tuple(np.median(a, 0)))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        step()
    pr.disable()
    ps = pstats.Stats(pr).sort_stats("tottime")
    ps.print_stats(25)


if __name__ == "__main__":
    main()
