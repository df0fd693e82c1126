"""Debug: two fused submissions back to back (engine level, NaN-filled waveform buffers) against
the two-call form; reports NaN (never written) and differing samples."""
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
eng = get_engine(dev)
B, r, pad = len(ids), 2, int(voc.inference_padding)
Tn = int(max(lens))
sub = x[:, :Tn].contiguous()


def two_calls(steps):
    a = taco.inference(x, text_lengths=lens, max_decoder_steps=steps)
    return voc.inference(a[1].transpose(1, 2), lengths=taco.last_mel_lengths.copy())


with torch.no_grad():
    ref = {"a": two_calls(steps_a), "b": two_calls(steps_b)}
    for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
        subs = {}
        for nm, steps in (("a", steps_a), ("b", steps_b)):
            S_cap = max(steps)
            outs = taco._out_tensors(B, S_cap, r, Tn, dev)
            wbuf = torch.full((B * voc.hop * (S_cap * r + 2 * pad),), float("nan"), device=dev)
            with eng.lock:
                st, _, ticket = eng.taco_mbmelgan_submit(sub, lens, r, np.asarray(steps), S_cap,
                                                         taco.decoder.stop_threshold, *outs, pad, wbuf)
            subs[nm] = (ticket, wbuf, outs, S_cap)
        for nm in ("a", "b"):
            eng.taco_mbmelgan_finish(subs[nm][0], dev)
        torch.cuda.synchronize()
        for nm in ("a", "b"):
            _, wbuf, outs, S_cap = subs[nm]
            L = voc.hop * (S_cap * r + 2 * pad)
            w = wbuf[:B * L].view(B, 1, L)
            u = ref[nm]
            nan = int(torch.isnan(w).sum())
            d = (w - u).abs()
            d[torch.isnan(d)] = 0
            n = int((d > 0).sum())
            msg = f"{trial} {nm}: nan {nan}, differ {n}, max {float(d.max()):.3e}"
            if n or nan:
                bad = torch.nonzero(((w - u).abs() > 0) | torch.isnan(w))
                rr, pp = int(bad[0, 0]), bad[bad[:, 0] == bad[0, 0], 2]
                msg += f" | row {rr} samples {pp[:20].tolist()} got {w[rr, 0, pp[:4]].tolist()} ref {u[rr, 0, pp[:4]].tolist()}"
                # the postnet output itself
                post = outs[1]
            print(msg, flush=True)
print("gemm mode, fallbacks:", eng.gemm_mode())
