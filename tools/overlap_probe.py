"""Probe: does running batch i's MB-MelGAN concurrently with batch i + 1's Tacotron2 (two library
contexts, two streams) shorten the C2 step? Not part of the library or the bench.
  python tools/overlap_probe.py [n]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from tts_amd._lib import Engine  # noqa: E402
from tts_amd.workload import forced_steps, lj_profile, pad_batch, synthetic_ids  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
MODE = sys.argv[3] if len(sys.argv) > 3 else "taco"
dev = torch.device("cuda", 0)
taco, tsd, voc, vsd, tcfg, vcfg = bench.build_models(dev)
taco.decoder.verbose = False
taco.decoder.set_r(2)
mine, my_T, my_prof, M_all = bench.rank_shard(1, 0, 32, 2)
T_prof, M_prof = lj_profile()
ids = synthetic_ids(T_prof)
batch, lens = pad_batch([ids[i] for i in my_prof])
batch_t = torch.from_numpy(batch).to(dev)
steps = forced_steps([M_all[i] for i in mine], 2)
engB = Engine(0)
voc._sync(engB)
pad = int(voc.inference_padding)


def taco_call():
    _, post, _, _ = taco.inference(batch_t, text_lengths=lens, max_decoder_steps=steps)
    return post, np.asarray(taco.last_mel_lengths, np.int64)


def voc_call(post, ml):
    c = post.transpose(1, 2)
    wav = torch.empty(c.shape[0], 1, 256 * (c.shape[2] + 2 * pad), device=dev)
    engB.melgan_infer(c, ml, pad, wav)
    return wav


def serial(k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        post, ml = taco_call()
        voc_call(post, ml)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / k


sV = torch.cuda.Stream(dev)


from concurrent.futures import ThreadPoolExecutor  # noqa: E402

ex = ThreadPoolExecutor(1)


def voc_on_sV(prev, ev):
    # the library's non-fused vocoder call waits for its range flag before returning, so it runs
    # on a worker thread (ctypes drops the GIL) while the main thread decodes the next batch
    with torch.cuda.stream(sV):
        sV.wait_event(ev)
        w = voc_call(*prev)
    prev[0].record_stream(sV)
    return w


def overlapped(k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    prev = None
    fut = None
    for i in range(k + 1):
        if prev is not None:  # batch i - 1's vocoder on its own stream, behind its decode
            if fut is not None:
                fut.result()
            ev = torch.cuda.Event()
            ev.record()
            fut = ex.submit(voc_on_sV, prev, ev)
        if i < k:
            prev = taco_call()
    fut.result()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / k


# correctness under overlap: every overlapped vocoder output against the serial one
post0, ml0 = taco_call()
ref = voc_call(post0, ml0).clone()
torch.cuda.synchronize()
bad = 0
for trial in range(int(sys.argv[2]) if len(sys.argv) > 2 else 10):
    ev = torch.cuda.Event()
    ev.record()
    fut = ex.submit(voc_on_sV, (post0, ml0), ev)
    if MODE == "vv":  # another vocoder beside it (the default context, its own workspace)
        c = post0.transpose(1, 2)
        wv = torch.empty(c.shape[0], 1, 256 * (c.shape[2] + 2 * pad), device=dev)
        voc.inference(c, lengths=ml0)
    elif MODE == "enc":  # only the Tacotron2 encoder (persistent BiLSTM) beside it, several times
        from tts_amd._lib import get_engine
        ea = get_engine(dev)
        eo = torch.empty(batch_t.shape[0], batch_t.shape[1], 512, device=dev)
        with ea.lock:
            for _ in range(6):
                ea.taco_encoder(batch_t, lens, eo)
    elif MODE == "dk":  # only the persistent decoder kernel (timing entry) beside it
        from tts_amd._lib import get_engine
        ea = get_engine(dev)
        with ea.lock:
            ea.time_decoder_kernel(1, 100)
    else:
        taco_call()  # a Tacotron2 call beside it (its own context and workspace)
    w = fut.result()
    torch.cuda.synchronize()
    d = (w - ref).abs()
    n = int((d > 0).sum())
    bad += n > 0
    print(f"trial {trial}: {n} values differ, max {float(d.max()):.3e}", flush=True)
print("overlapped vocoder outputs differing:", bad)
