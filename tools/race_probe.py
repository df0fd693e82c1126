"""Probe: which MB-MelGAN stage goes wrong when a persistent encoder BiLSTM (another library context)
runs beside it (profiles/r06/v23_voc_overlap_rejected.txt). Each trial runs one stage on engine B
(worker thread, own stream) while the main thread runs encoder calls on the default engine, and
compares the stage's output with the same stage run alone.

    python tools/race_probe.py <trials> <stage>[,<stage>...]
stages: gen (generator bands, output conv unfused), wav (fused output conv + PQMF), pqmf (PQMF
synthesis of the reference bands), wavf32 (wav with fp32 GEMMs)."""
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from tts_amd._lib import Engine, get_engine  # noqa: E402
from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids  # noqa: E402

trials = int(sys.argv[1]) if len(sys.argv) > 1 else 10
stages = (sys.argv[2] if len(sys.argv) > 2 else "gen,wav,pqmf").split(",")
dev = torch.device("cuda", 0)
taco, _, voc, _, _, _ = bench.build_models(dev)
taco.decoder.verbose = False
taco.decoder.set_r(2)
mine, my_T, my_prof, M_all = bench.rank_shard(1, 0, 32, 2)
T_prof, _ = lj_profile()
ids = synthetic_ids(T_prof)
batch, lens = pad_batch([ids[i] for i in my_prof])
batch_t = torch.from_numpy(batch).to(dev)
steps = forced_steps([M_all[i] for i in mine], 2)
_, post, _, _ = taco.inference(batch_t, text_lengths=lens, max_decoder_steps=steps)
ml = np.asarray(taco.last_mel_lengths, np.int64)
c = post.transpose(1, 2).contiguous()
B, _, M = c.shape
pad = int(voc.inference_padding)
up = int(np.prod(voc.cfg.upsample_factors))
Ls = up * (M + 2 * pad)
G = voc.pqmf_layer.G.to(dev, torch.float32).reshape(4, -1).contiguous()
engB = Engine(0)
voc._sync(engB)
ea = get_engine(dev)
sV = torch.cuda.Stream(dev)
ex = ThreadPoolExecutor(1)


def run(stage, src=None):
    if stage == "gen":
        out = torch.full((B, 4, Ls), float("nan"), device=dev)
        engB.melgan_generator(c, ml, pad, out)
    elif stage == "pqmf":
        out = torch.full((B, 1, 4 * Ls), float("nan"), device=dev)
        engB.pqmf_synthesis(src, G, out)
    else:
        out = torch.full((B, 1, 4 * Ls), float("nan"), device=dev)
        engB.melgan_infer(c, ml, pad, out)
    return out


def on_sV(stage, src, ev):
    with torch.cuda.stream(sV):
        sV.wait_event(ev)
        w = run(stage, src)
        sV.synchronize()
    return w


def describe(d, stage):
    idx = torch.nonzero(d > 0).cpu().numpy()
    rows = sorted(set(idx[:, 0].tolist()))
    if stage == "gen":  # (row, band, position)
        bands = sorted(set(idx[:, 1].tolist()))
        pos = idx[:, 2]
        return f"rows {rows[:8]} bands {bands} pos {pos.min()}..{pos.max()} first {idx[:6, 1:].tolist()}"
    pos = idx[:, 2]
    ph = sorted(set((pos % 4).tolist()))
    return f"rows {rows[:8]} phases {ph} pos {pos.min()}..{pos.max()} first {pos[:12].tolist()}"


bands_ref = run("gen")
torch.cuda.synchronize()
for stage in stages:
    if stage == "wavf32":
        engB.set_gemm_mode("f32")
        st = "wav"
    else:
        engB.set_gemm_mode("x3")
        st = stage
    ref = run(st, bands_ref).clone()
    torch.cuda.synchronize()
    assert not torch.isnan(ref).any(), stage
    bad = 0
    for trial in range(trials):
        ev = torch.cuda.Event()
        ev.record()
        fut = ex.submit(on_sV, st, bands_ref, ev)
        eo = torch.empty(batch_t.shape[0], batch_t.shape[1], 512, device=dev)
        with ea.lock:
            for _ in range(6):
                ea.taco_encoder(batch_t, lens, eo)
        w = fut.result()
        torch.cuda.synchronize()
        nan = int(torch.isnan(w).sum())
        d = (w - ref).abs().nan_to_num(0.0)
        n = int((d > 0).sum())
        bad += (n > 0) or (nan > 0)
        msg = f"{stage} trial {trial}: {n} differ, max {float(d.max()):.3e}, nan {nan}"
        if n:
            msg += " | " + describe(d, st)
        print(msg, flush=True)
    print(f"== {stage}: {bad} / {trials} trials differ", flush=True)
engB.set_gemm_mode("x3")
