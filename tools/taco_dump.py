"""Tacotron2 outputs (bench.py's random-init C2 model, the first 12 LJ-profile utterances, forced
lengths at r = 2) saved to an .npz file, for bit-identity checks between library settings run in
separate processes (e.g. TTS_BAR_CALIBRATE=0 / 1: the decoder's barrier blocks picked by timing or
taken in order; the barrier's place must not change a single bit).

    python tools/taco_dump.py out.npz [n]     (n utterances, default 12; > 32 repeats the profile)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids  # noqa: E402


def main(path, n=12):
    dev = torch.device("cuda", 0)
    taco, _, _, _, _, _ = bench.build_models(dev)
    taco.decoder.verbose = False
    taco.decoder.set_r(2)
    T, M = lj_profile()
    T, M = (list(T) * 2)[:n], (list(M) * 2)[:n]
    batch, lens = pad_batch(synthetic_ids(T))
    dec, post, align, stop = taco.inference(torch.from_numpy(batch).to(dev), text_lengths=lens,
                                            max_decoder_steps=forced_steps(M, 2))
    np.savez(path, dec=dec.cpu().numpy(), post=post.cpu().numpy(), align=align.cpu().numpy(),
             stop=stop.cpu().numpy(), steps=np.asarray(taco.last_steps))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
