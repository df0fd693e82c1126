"""Host-side cost of one bench step (Python + ctypes + HIP enqueue) beside its wall time: cProfile
over 5 steps of the bench workload, sorted by own time. Not part of the library.
  python tools/host_prof.py"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    taco, tsd, voc, vsd, tcfg, vcfg = bench.build_models(dev)
    taco.decoder.set_r(2)
    taco.decoder.verbose = False
    T_prof, M_prof = bench.lj_profile()
    ids = bench.synthetic_ids(T_prof)
    steps = bench.forced_steps(M_prof, 2)
    batch, lens = bench.pad_batch(ids)
    batch_t = torch.from_numpy(batch).to(dev)

    def one():
        _, post, _, _ = taco.inference(batch_t, text_lengths=lens, max_decoder_steps=steps)
        return voc.inference(post.transpose(1, 2), lengths=taco.last_mel_lengths)

    for _ in range(2):
        one()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(5):
        one()
    torch.cuda.synchronize()
    pr.disable()
    print(f"wall per step {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms")
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
