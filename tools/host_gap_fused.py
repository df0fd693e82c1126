"""Host-side intervals of the C2 bench step on the fused entry (Tacotron2.inference_vocoded ->
tts_taco_mbmelgan_infer): medians over N steps of
  c_us       the library call (C++ preparation, enqueue, both models' GPU work, status and range-flag
             read-backs)
  py_us      the rest of the step (Python around the call: argument preparation, output tensors,
             outputs' assembly)
  step_us    wall time per step (perf_counter; the call ends synchronised)
plus the same for the two-call form. Not part of the library: python tools/host_gap_fused.py [steps]"""
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
    x = torch.from_numpy(batch).to(dev)
    steps = forced_steps(M_prof, 2)
    eng = get_engine(dev)
    stamps = []
    orig = {k: getattr(eng, k) for k in ("taco_mbmelgan_infer", "taco_infer", "melgan_infer")}

    def wrap(name):
        def f(*a, **k):
            t0 = time.perf_counter()
            r = orig[name](*a, **k)
            stamps.append((name, t0, time.perf_counter()))
            return r
        return f

    for k in orig:
        setattr(eng, k, wrap(k))
    res = {}
    for form in ("fused", "two_calls"):
        def step():
            if form == "fused":
                taco.inference_vocoded(x, voc, text_lengths=lens, max_decoder_steps=steps)
            else:
                _, post, _, _ = taco.inference(x, text_lengths=lens, max_decoder_steps=steps)
                voc.inference(post.transpose(1, 2), lengths=taco.last_mel_lengths)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        c, st = [], []
        for _ in range(n):
            stamps.clear()
            t0 = time.perf_counter()
            step()
            t1 = time.perf_counter()
            st.append(t1 - t0)
            c.append(sum(e - s for _, s, e in stamps))
        res[form] = {"step_us": round(float(np.median(st)) * 1e6, 1), "c_us": round(float(np.median(c)) * 1e6, 1),
                     "py_us": round(float(np.median(np.array(st) - np.array(c))) * 1e6, 1)}
    print(res)


if __name__ == "__main__":
    main()
