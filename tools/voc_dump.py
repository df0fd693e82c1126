"""MB-MelGAN output saved to an .npy file, for bit-identity checks between library modes run in
separate processes (e.g. TTS_CT_FUSE=0 / 1: the last ConvTranspose fused into the C = 48 stack
kernel or launched on its own). Default: a seeded ragged batch of 5 random mels; --bench: the C2
bench batch (bench.py's Tacotron2 mels).

    python tools/voc_dump.py out.npy [--bench]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids  # noqa: E402


def main(path, full):
    dev = torch.device("cuda", 0)
    taco, _, voc, _, _, _ = bench.build_models(dev)
    if full:
        taco.decoder.verbose = False
        T, M = lj_profile()
        batch, lens = pad_batch(synthetic_ids(T))
        taco.decoder.set_r(2)
        _, post, _, _ = taco.inference(torch.from_numpy(batch).to(dev), text_lengths=lens,
                                       max_decoder_steps=forced_steps(M, 2))
        mel, mlens = post.transpose(1, 2), taco.last_mel_lengths
    else:
        mlens = np.array([37, 120, 5, 64, 91])
        mel = torch.from_numpy(np.random.RandomState(3).randn(5, 80, 120).astype(np.float32)).to(dev)
    wav = voc.inference(mel, lengths=mlens)
    np.save(path, wav.cpu().numpy())
    print(path, tuple(wav.shape), float(wav.abs().max()))


if __name__ == "__main__":
    main(sys.argv[1], "--bench" in sys.argv[2:])
