"""Benchmark: Tacotron2-DDC + MultiBand-MelGAN inference, batch 32 LJ-length utterances per GPU.

One "step" = Tacotron2.inference on the rank's 32-utterance batch (encoder, graph-captured
autoregressive decoder, postnet) followed by MultibandMelganGenerator.inference on the
resulting mels (generator + PQMF). Forced lengths: stop bias -1e4 and
max_decoder_steps_i = ceil(M_i / r), so every run does exactly the same work.

Prints ONE JSON line (rank 0). ``value`` = mel frames produced per second by the whole
pipeline over all ranks; Tacotron2-only frames/s and end-to-end RTF are extra fields.
Launch for N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tts_amd import MultibandMelganGenerator, Tacotron2  # noqa: E402
from tts_amd.spec import MelganConfig, TacotronConfig, melgan_spec, tacotron2_spec  # noqa: E402
from tts_amd.weights import synth_state_dict  # noqa: E402
from tts_amd.workload import (HOP, SAMPLE_RATE, forced_steps, lj_profile, pad_batch,  # noqa: E402
                              replicated_workload, synthetic_ids)

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
F32_PEAK_TFLOPS = 157.3     # dense fp32 (vector == f32 MFMA rate)
F16_PEAK_TFLOPS = 2500.0    # dense f16 MFMA (v_mfma_f32_16x16x32_f16)
X3_PEAK_TFLOPS = F16_PEAK_TFLOPS / 3  # fp32-equivalent rate of the split-f16 form (3 f16 MFMAs per product)


def build_models(device, seed=0):
    tcfg = TacotronConfig()
    tsd = synth_state_dict(tacotron2_spec(tcfg), seed)
    tsd["decoder.stopnet.1.linear_layer.bias"] = np.array([-1e4], np.float32)  # forced length
    taco = Tacotron2(num_chars=tcfg.num_chars, num_speakers=0, r=tcfg.r, attn_norm=tcfg.attn_norm,
                     double_decoder_consistency=True, ddc_r=tcfg.ddc_r)
    taco.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in tsd.items()})
    taco = taco.to(device).eval()
    vcfg = MelganConfig()
    vsd = synth_state_dict(melgan_spec(vcfg, weight_norm=True), seed + 1)
    voc = MultibandMelganGenerator(in_channels=80, out_channels=4, base_channels=384,
                                   upsample_factors=vcfg.upsample_factors, num_res_blocks=vcfg.num_res_blocks)
    full = voc.state_dict()
    for k, v in vsd.items():
        full[k] = torch.from_numpy(v)
    voc.load_state_dict(full)
    voc.remove_weight_norm()
    voc.inference_padding = 0      # as TTS/server/synthesizer.py:86
    voc = voc.to(device).eval()
    return taco, tsd, voc, vsd, tcfg, vcfg


def cpu_baseline(tsd, vsd, tcfg, vcfg, ids, steps, r, budget_s):
    """Oracle (numpy fp32 restatement) at B=1 per utterance, like the reference CPU path."""
    from threadpoolctl import threadpool_limits
    from oracle.melgan_np import MelganOracle
    from oracle.taco_np import TacoOracle
    from tts_amd.pqmf import pqmf_filters
    from tts_amd.spec import melgan_layers
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cores = max(1, min(cores, os.cpu_count() or 1))
    to = TacoOracle(tsd, tcfg.attn_norm, tcfg.r)
    vo = MelganOracle(vsd, melgan_layers(vcfg), pqmf_filters()[1])
    frames = 0
    n = 0
    with threadpool_limits(limits=cores):
        # warm-up on the shortest utterance (excluded, as SURVEY §8d asks)
        j = int(np.argmin(steps))
        _, p, _, _ = to.inference(ids[j], r, min(steps[j], 4))
        t0 = time.perf_counter()
        for i in range(len(ids)):
            _, p, _, _ = to.inference(ids[i], r, steps[i])
            vo.inference(p.T, pad=0)
            frames += p.shape[0]
            n += 1
            if time.perf_counter() - t0 > budget_s:
                break
        el = time.perf_counter() - t0
    audio = frames * HOP / SAMPLE_RATE
    return {"value": frames / el, "unit": "mel-frames/s", "cores": cores, "kind": "port",
            "rtf": el / audio,
            "sample": f"first {n} of {len(ids)} LJ-profile utterances, B=1 sequential, r={r}, forced length "
                      f"({frames} frames), numpy fp32 oracle + MB-MelGAN oracle, {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--r", type=int, default=2)
    ap.add_argument("--per-gpu-batch", type=int, default=32)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--f32-steps", type=int, default=3, help="steps re-timed with fp32-MFMA GEMMs only (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    taco, tsd, voc, vsd, tcfg, vcfg = build_models(dev)
    r = args.r
    taco.decoder.set_r(r)
    taco.decoder.verbose = False  # forced lengths end every utterance at max_decoder_steps
    T_all, M_all, shards = replicated_workload(world, args.per_gpu_batch)
    mine = shards[rank]
    T_prof, M_prof = lj_profile()
    ids = synthetic_ids(T_prof)              # C3 replicates the same 32 utterances
    my_ids = [ids[i % len(ids)] for i in mine]
    steps = forced_steps([M_all[i] for i in mine], r)
    batch, lens = pad_batch(my_ids)
    batch_t = torch.from_numpy(batch).to(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tt, tv = [], []

    def one_step(record):
        if record:
            ev[0].record()
        _, post, _, _ = taco.inference(batch_t, text_lengths=lens, max_decoder_steps=steps)
        if record:
            ev[1].record()
        mel_lens = taco.last_mel_lengths
        wav = voc.inference(post.transpose(1, 2), lengths=mel_lens)  # read in place (tts_melgan_infer_strided)
        if record:
            ev[2].record()
            torch.cuda.synchronize()
            tt.append(ev[0].elapsed_time(ev[1]))
            tv.append(ev[1].elapsed_time(ev[2]))
        return int(mel_lens.sum()), wav

    for _ in range(args.warmup):
        one_step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    frames = 0
    for _ in range(args.steps):
        f, _ = one_step(False)
        frames += f
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    per_step_frames = frames // args.steps
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        fr = torch.tensor([per_step_frames], device=dev, dtype=torch.float64)
        dist.all_reduce(fr, op=dist.ReduceOp.SUM)
        per_step_frames = int(fr.item())
    ms_step = el / args.steps * 1000.0
    value = per_step_frames / (ms_step / 1000.0)
    audio_s = per_step_frames * HOP / SAMPLE_RATE
    # per-stage split (separate, event-timed passes after the timed region)
    for _ in range(2):
        one_step(True)
    taco_ms, voc_ms = float(np.median(tt)), float(np.median(tv))
    my_frames = int(sum(s * r for s in steps))

    from tts_amd._lib import get_engine
    eng = get_engine(dev)
    gemm_mode, fallbacks = eng.gemm_mode()
    # decoder launch stats of the last step above (the headline GEMM mode), before the fp32 pass
    path, launches = eng.decoder_stats()
    # the same step with every GEMM on the fp32 MFMA (no split-f16 kernels), for comparison
    f32_ms = None
    if gemm_mode == "x3" and args.f32_steps > 0:
        eng.set_gemm_mode("f32")
        one_step(False)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.f32_steps):
            one_step(False)
        torch.cuda.synchronize()
        f32_ms = (time.perf_counter() - t1) / args.f32_steps * 1000.0
        eng.set_gemm_mode("x3")

    # dominant decoder kernel, timed live with HIP events on the library's stream (stats above)
    if path == 1:
        # persistent decoder: the MT = 2 launch (32-row batch tile) carries most steps. Algorithmic
        # work = useful row-steps (rows still decoding) x the per-row GEMM flops of one step
        ms0, st0 = launches[0]
        flop_row = 2 * (4096 * 2560          # decoder_rnn [W_ih | W_hh]
                        + 4096 * 1536        # attention_rnn ctx/h part
                        + 4096 * 256         # attention_rnn prenet part
                        + (1 + 80 * r) * 1536  # projection (r frames) + stopnet
                        + 80 * 256 + 256 * 256  # prenet
                        + 1024 * 128)        # query projection
        row_steps = sum(min(s_, st0) for s_ in steps[:16 * ((len(mine) + 15) // 16)])
        flops = row_steps * flop_row
        achieved = flops / (ms0 * 1e-3) / 1e12
        step_ms = ms0 / max(st0, 1)
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "persist_pmc.json")
        if os.path.exists(pmc):
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        # split-f16 mode: the decoder's GEMM parts run 3 f16 MFMAs per fp32 product, so the
        # ceiling is the f16 MFMA peak / 3 in fp32-equivalent FLOP/s; fp32 mode: the fp32 MFMA peak
        peak = X3_PEAK_TFLOPS if gemm_mode == "x3" else F32_PEAK_TFLOPS
        roof = {"kernel": "persist_decoder_kernel<2%s> (whole decoder loop, weights resident on chip)"
                          % (", split-f16" if gemm_mode == "x3" else ""),
                "bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "frac_vs_fp32_mfma_peak": round(achieved / F32_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "avg_launch_us": round(ms0 * 1000.0, 1), "algorithmic_flops": flops,
                "launch_steps": st0, "launches": [[round(m_, 3), s_] for m_, s_ in launches]}
    else:
        k4_ms = eng.time_decoder_kernel(0, args.kernel_iters)
        step_ms = eng.time_decoder_kernel(1, max(4, args.kernel_iters // 8))
        Bp = 16 * ((len(mine) + 15) // 16)
        k4_bytes = 4 * (4096 * 2560                         # decoder_rnn [W_ih | W_hh], gate-interleaved tiles
                        + 4096                              # folded biases
                        + Bp * 2560                         # activations read [h_att | ctx | h_dec]
                        + Bp * 1024 * 3)                    # c read/write, h write
        achieved = k4_bytes / (k4_ms * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "k4_pmc.json")
        if os.path.exists(pmc):
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        roof = {"kernel": "decoder K4 (decoder_rnn LSTMCell: K=2560 skinny GEMM + fused cell update)",
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "avg_launch_us": round(k4_ms * 1000.0, 2), "algorithmic_bytes": k4_bytes}

    out = {
        "metric": "mel-frames/s (Tacotron2-DDC + MB-MelGAN end-to-end)",
        "value": round(value, 1),
        "unit": "mel-frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "gemm": ("split-f16 MFMA, fp32-accurate (split16.h: 3 f16 products per fp32 product, fp32 accumulate)"
                 if gemm_mode == "x3" else "fp32 MFMA"),
        "f32_gemm_ms_per_step": None if f32_ms is None else round(f32_ms, 3),
        "x3_range_fallbacks": fallbacks,
        "data": "synthetic (LJ-profile lengths, RandomState(0) ids, seeded random weights, forced length)",
        "config": {"workload": f"C{2 if world == 1 else 3}: Tacotron2-DDC (r_init=7, r={r}, sigmoid attn) + "
                               f"MB-MelGAN [8,4,2]x4, {args.per_gpu_batch} LJ-length utterances per GPU",
                   "global_batch": args.per_gpu_batch * world, "r": r, "parallelism": f"replicas x{world}"},
        "e2e_rtf": ms_step / 1000.0 / audio_s,
        "tacotron2_mel_frames_per_s": round(my_frames / (taco_ms / 1000.0) * world, 1),
        "tacotron2_ms": round(taco_ms, 3),
        "vocoder_ms": round(voc_ms, 3),
        "decoder_step_us": round(step_ms * 1000.0, 2),
        "decoder_steps": int(max(steps)),
        "decoder_path": "persistent" if path == 1 else "step-graphs",
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(tsd, vsd, tcfg, vcfg, ids, forced_steps(M_prof, r), r,
                                           args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
