"""Debug: fused submissions back to back against the two-call form (tests/test_gpu_parity.py
test_fused_submit_pipelined_and_short_decode's first part), with the size of any difference."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import bench  # noqa: E402
from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids  # noqa: E402
from tts_amd._lib import get_engine  # noqa: E402

dev = torch.device("cuda", 0)
taco, tsd, voc, vsd, tcfg, vcfg = bench.build_models(dev)
taco.decoder.set_r(2)
taco.decoder.verbose = False
T_prof, M_prof = lj_profile()
ids = synthetic_ids(T_prof)
batch, lens = pad_batch(ids)
x = torch.from_numpy(batch).to(dev)
full = forced_steps(M_prof, 2)
steps_a = [max(3, s_ // 5) for s_ in full]
steps_b = [max(3, s_ // 7) for s_ in full][::-1]


def two_calls(steps):
    a = taco.inference(x, text_lengths=lens, max_decoder_steps=steps)
    return a + (voc.inference(a[1].transpose(1, 2), lengths=taco.last_mel_lengths.copy()),)


eng = get_engine(dev)
with torch.no_grad():
    ref_a, ref_b = two_calls(steps_a), two_calls(steps_b)
    for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        f0 = eng.x3_fallbacks() if hasattr(eng, "x3_fallbacks") else None
        fa = taco.inference_vocoded_submit(x, voc, text_lengths=lens, max_decoder_steps=steps_a)
        fb = taco.inference_vocoded_submit(x, voc, text_lengths=lens, max_decoder_steps=steps_b)
        got_a, got_b = fa.result(), fb.result()
        torch.cuda.synchronize()
        for nm, ref, got in (("a", ref_a, got_a), ("b", ref_b, got_b)):
            for k, (u, v) in enumerate(zip(ref, got)):
                if u.shape != v.shape:
                    print(trial, nm, k, "shape", u.shape, v.shape)
                    continue
                d = (u - v).abs()
                n = int((d > 0).sum())
                if n:
                    rows = sorted(set(int(i) for i in torch.nonzero(d.reshape(d.shape[0], -1) > 0)[:, 0].tolist()))
                    print(trial, nm, k, "differ", n, "of", d.numel(), "max", float(d.max()), "rows", rows[:10], flush=True)
                    dd = d.reshape(d.shape[0], -1)
                    r0 = rows[0]
                    pos = torch.nonzero(dd[r0] > 0)[:, 0]
                    L = int(taco.last_mel_lengths[r0]) if False else -1
                    print("   row", r0, "positions", int(pos.min()), "..", int(pos.max()), "count", int(pos.numel()),
                          "row length", dd.shape[1], flush=True)
                else:
                    print(trial, nm, k, "equal", flush=True)
