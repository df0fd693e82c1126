"""Host-side intervals of the C2 bench step: where the ~0.25 ms between the end of
the Tacotron2 kernels and the start of the vocoder's goes. Wraps the engine's C-ABI calls with
perf_counter stamps and reports medians over N steps:
  taco_c      the tts_taco_infer call (enqueue, the GPU work, the status read-back)
  py_between  from its return to the tts_melgan_infer_strided call (Python: Tacotron2.inference's
              post-processing, bench's one_step, MultibandMelganGenerator.inference's checks)
  voc_c       the vocoder call (enqueue, GPU work, range-flag read-back)
Not part of the library: python tools/host_gap.py [steps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tts_amd._lib import get_engine  # noqa: E402
from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    taco, _, voc, _, _, _ = bench.build_models(dev)
    taco.decoder.verbose = False
    taco.decoder.set_r(2)
    T_prof, M_prof = lj_profile()
    batch, lens = pad_batch(synthetic_ids(T_prof))
    batch_t = torch.from_numpy(batch).to(dev)
    steps = forced_steps(M_prof, 2)
    eng = get_engine(dev)
    stamps = {}
    orig_t, orig_v = eng.taco_infer, eng.melgan_infer

    def taco_w(*a, **k):
        stamps["t0"] = time.perf_counter()
        out = orig_t(*a, **k)
        stamps["t1"] = time.perf_counter()
        return out

    def voc_w(*a, **k):
        stamps["v0"] = time.perf_counter()
        out = orig_v(*a, **k)
        stamps["v1"] = time.perf_counter()
        return out

    eng.taco_infer, eng.melgan_infer = taco_w, voc_w
    rec = []
    for i in range(n + 2):
        torch.cuda.synchronize()
        s0 = time.perf_counter()
        _, post, _, _ = taco.inference(batch_t, text_lengths=lens, max_decoder_steps=steps)
        wav = voc.inference(post.transpose(1, 2), lengths=taco.last_mel_lengths)
        torch.cuda.synchronize()
        s1 = time.perf_counter()
        if i >= 2:
            rec.append([(stamps["t0"] - s0) * 1e6, (stamps["t1"] - stamps["t0"]) * 1e6,
                        (stamps["v0"] - stamps["t1"]) * 1e6, (stamps["v1"] - stamps["v0"]) * 1e6,
                        (s1 - stamps["v1"]) * 1e6, (s1 - s0) * 1e6])
    med = np.median(np.array(rec), axis=0)
    names = ["py_before_taco", "taco_c", "py_between", "voc_c", "py_after", "step"]
    print("{" + ", ".join(f'"{k}_us": {v:.1f}' for k, v in zip(names, med)) + "}")
    del wav




def profile(n=10):
    """cProfile of n steps' host code (the C calls show as two leaf entries)."""
    import cProfile
    import pstats
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    taco, _, voc, _, _, _ = bench.build_models(dev)
    taco.decoder.verbose = False
    taco.decoder.set_r(2)
    T_prof, M_prof = lj_profile()
    batch, lens = pad_batch(synthetic_ids(T_prof))
    batch_t = torch.from_numpy(batch).to(dev)
    steps = forced_steps(M_prof, 2)

    def step():
        _, post, _, _ = taco.inference(batch_t, text_lengths=lens, max_decoder_steps=steps)
        return voc.inference(post.transpose(1, 2), lengths=taco.last_mel_lengths)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    rows = sorted(((v[2], v[3], v[1], k) for k, v in st.stats.items()), reverse=True)[:40]
    for tt, ct, nc, k in rows:
        print(f"{tt * 1e6 / n:9.1f} us/step self {ct * 1e6 / n:10.1f} us/step cum {nc / n:5.1f} calls  {k[0].split('/')[-1]}:{k[1]}({k[2]})")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "prof":
        profile(int(sys.argv[1]))
    else:
        main()
