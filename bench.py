"""Benchmark: Tacotron2-DDC + MultiBand-MelGAN inference, batch 32 LJ-length utterances per GPU.

One "step" = Tacotron2.inference on the rank's 32-utterance batch (encoder, persistent
autoregressive decoder, postnet) followed by MultibandMelganGenerator.inference on the
resulting mels (generator + PQMF), as ONE library submission (Tacotron2.inference_vocoded_submit ->
tts_taco_mbmelgan_submit / _finish; bit-identical to the two calls). The timed loop keeps the host
one batch ahead: batch i + 1 is submitted (its Tacotron2 runs beside batch i's vocoder, which the
library keeps on a second stream) before batch i's waveforms are taken, and every batch is
finished inside the timed region; the blocking one-call and two-call
forms are timed beside it. Forced lengths: stop bias -1e4 and
max_decoder_steps_i = ceil(M_i / r), so every run does exactly the same work.

Prints ONE JSON line (rank 0). ``value`` = mel frames produced per second by the whole
pipeline over all ranks, ids and waveforms resident in HBM (r = 2). Extra fields:
Tacotron2-only frames/s, end-to-end RTF, ``e2e_rtf_host`` (ids on the host -> per-utterance
waveforms on the host), the r = 1 run (``r1``), and ``roofline.pipeline_frac`` =
SURVEY 8d's whole-pipeline bound / measured.
Launch for N > 1: ``python bench.py --gpus N`` starts N ranks itself (torch.distributed.run as a
child process, before any GPU call; launch_plan), or run it as the ranks of
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`` (WORLD_SIZE must equal N).
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
from tts_amd.multigpu import shard_plan  # noqa: E402
from tts_amd.workload import (HOP, SAMPLE_RATE, forced_steps, lj_profile, pad_batch,  # noqa: E402
                              replicated_workload, synthetic_ids)

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
F32_PEAK_TFLOPS = 157.3     # dense fp32 (vector == f32 MFMA rate)
F16_PEAK_TFLOPS = 2500.0    # dense f16 MFMA (v_mfma_f32_16x16x32_f16)
X3_PEAK_TFLOPS = F16_PEAK_TFLOPS / 3  # fp32-equivalent rate of the split-f16 form (3 f16 MFMAs per product)

# SURVEY.md 8d algorithmic work (checked there against torch.utils.flop_counter on the reference)
DEC_FLOP_ROW_STEP = 37_809_248     # prenet, both LSTMCells, query, projection at r_init = 7, stopnet
ATT_FLOP_PER_T = 13_440            # loc-conv 3,968 + loc-dense 8,192 + v 256 + context 1,024 per position
DEC_W_BYTES = 75_711_112           # 18,927,778 fp32 decoder parameters read per batched step
ENC_FLOP_TOKEN = 11_010_048 + 131_072   # 3 convs + BiLSTM, + processed_inputs
POST_FLOP_FRAME = 8_683_520
VOC_FLOP_FRAME = 36_128_768        # MB-MelGAN generator + PQMF


def pipeline_bound_ms(T, steps, r, peak_tflops=F32_PEAK_TFLOPS):
    """SURVEY 8d lower bound for one batch: decoder sum over steps of max(bytes / HBM, flops / peak)
    with the active set shrinking as utterances finish, plus encoder + postnet + vocoder flops / peak.
    Returns (total_ms, decoder_ms). 10.15 ms at r=2 and 14.59 ms at r=1 for the C2 batch."""
    T = np.asarray(T, np.float64)
    st = np.asarray(steps)
    dec = 0.0
    for s_ in range(int(st.max())):
        a = st > s_
        fl = (DEC_FLOP_ROW_STEP + ATT_FLOP_PER_T * T[a]).sum()
        by = DEC_W_BYTES + (2580.0 * T[a] + 320.0 * r + 37_500.0).sum()  # inputs+keys+alpha, align, frames, states
        dec += max(by / (HBM_PEAK_GBS * 1e9), fl / (peak_tflops * 1e12))
    frames = float((st * r).sum())
    other = (T.sum() * ENC_FLOP_TOKEN + frames * (POST_FLOP_FRAME + VOC_FLOP_FRAME)) / (peak_tflops * 1e12)
    return (dec + other) * 1e3, dec * 1e3


def latest_profile(name):
    """The newest record ``profiles/r<NN>/<name>`` (the current round's measurement of this tree
    once it exists), else ``profiles/<name>``; None if neither exists."""
    import glob
    rounds = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", name)), reverse=True)
    if rounds:
        return rounds[0]
    flat = os.path.join(ROOT, "profiles", name)
    return flat if os.path.exists(flat) else None


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


def cpu_facts():
    """Host CPU share as this process sees it: the affinity mask, and the physical cores behind it
    (distinct (physical id, core id) pairs of /proc/cpuinfo)."""
    aff = sorted(os.sched_getaffinity(0))
    core_of, model = {}, None
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            if ":" not in line:
                if "processor" in cur:
                    core_of[int(cur["processor"])] = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
                cur = {}
                continue
            k, v = (x.strip() for x in line.split(":", 1))
            cur[k] = v
            if k == "model name" and model is None:
                model = v
        if "processor" in cur:
            core_of[int(cur["processor"])] = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
    except OSError:
        pass
    phys = len({core_of[c] for c in aff if c in core_of}) or None
    return {"affinity_cpus": len(aff), "physical_cores_in_affinity": phys, "machine_cpus": os.cpu_count(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "model": model}


def cpu_baseline(tsd, vsd, tcfg, vcfg, ids, steps, r, budget_s):
    """The reference CPU path's op sequence (oracle/torch_cpu.py: PyTorch-CPU ATen restatement, SURVEY
    8d) at B=1 per utterance, Tacotron2 then MB-MelGAN, on the host's cores. Timed beside the imported
    reference in the build container by tools/cpu_baseline_check.py (profiles/r03/).
    The thread count is the CPU's best: torch.set_num_threads over {1, 2, 4, 8, 16} (capped by the
    affinity mask) on one short utterance, then the whole batch at the fastest setting, utterance by
    utterance until ``budget_s`` of CPU work."""
    from oracle.torch_cpu import MelganTorchCPU, TacoTorchCPU
    from tts_amd.pqmf import pqmf_filters
    from tts_amd.spec import melgan_layers
    facts = cpu_facts()
    cap = max(1, facts["affinity_cpus"])
    prev = torch.get_num_threads()
    sweep = {}
    try:
        to = TacoTorchCPU(tsd, tcfg.attn_norm, tcfg.r)
        vo = MelganTorchCPU(vsd, melgan_layers(vcfg), pqmf_filters()[1])
        j = int(np.argmin(steps))  # the shortest utterance: warm-up and thread sweep
        for nt in [n for n in (1, 2, 4, 8, 16) if n <= cap]:
            torch.set_num_threads(nt)
            _, p, _, _ = to.inference(ids[j], r, min(steps[j], 4))  # warm-up at this setting (excluded)
            vo.inference(p.T, pad=0)
            t0 = time.perf_counter()
            _, p, _, _ = to.inference(ids[j], r, steps[j])
            vo.inference(p.T, pad=0)
            sweep[nt] = round(p.shape[0] / (time.perf_counter() - t0), 1)
        cores = max(sweep, key=sweep.get)
        torch.set_num_threads(cores)
        frames = n = 0
        t_taco = t_voc = 0.0
        while n < len(ids) and t_taco + t_voc < budget_s:
            t0 = time.perf_counter()
            _, p, _, _ = to.inference(ids[n], r, steps[n])
            t1 = time.perf_counter()
            vo.inference(p.T, pad=0)
            t_voc += time.perf_counter() - t1
            t_taco += t1 - t0
            frames += p.shape[0]
            n += 1
    finally:
        torch.set_num_threads(prev)
    el = t_taco + t_voc
    audio = frames * HOP / SAMPLE_RATE
    calib = None  # this restatement timed beside the imported reference (build container, same weights)
    cpath = latest_profile(f"cpu_baseline_check_r{r}.json")
    if cpath:
        try:
            cj = json.load(open(cpath))
            calib = {"port_over_reference_e2e": cj["aten_port_over_reference_e2e"],
                     "port_vs_reference_post_max_abs": cj["aten_port_vs_reference_post_max_abs"],
                     "threads": cj["threads"], "source": os.path.relpath(cpath, ROOT)}
        except Exception:
            calib = None
    return {"value": round(frames / el, 1), "unit": "mel-frames/s", "cores": cores, "kind": "port",
            "rtf": el / audio, "tacotron2_mel_frames_per_s": round(frames / t_taco, 1), "calibration": calib,
            "thread_sweep_frames_per_s": sweep, "host": facts,
            "sample": f"{'all' if n == len(ids) else 'first'} {n} of {len(ids)} LJ-profile utterances, B=1 "
                      f"sequential, r={r}, forced length ({frames} frames): Tacotron2 {t_taco:.1f} s + MB-MelGAN "
                      f"{t_voc:.1f} s, PyTorch-CPU restatement of the reference op sequence (oracle/torch_cpu.py), "
                      f"{cores} threads (the fastest of the sweep on utterance {j}, {steps[j] * r} frames)"}


def rank_shard(world, rank, per_gpu_batch, r):
    """This rank's share of the global batch (C2 at world 1, C3 above: the 32-utterance LJ profile
    once per rank) through the product entry point's plan (tts_amd.multigpu.shard_plan: LPT on the
    decoder step counts, the token count breaking ties, no data-path collective). Returns the global
    indices of the rank's utterances, their token counts and their profile indices (ids come from
    synthetic_ids over the profile)."""
    T_all, M_all, _ = replicated_workload(world, per_gpu_batch)
    mine = shard_plan([s_ * 1e6 + t_ for s_, t_ in zip(forced_steps(M_all, r), T_all)], world)[rank]
    n_prof = len(lj_profile()[0])
    return mine, [T_all[i] for i in mine], [i % n_prof for i in mine], M_all


def aggregate(el_s, frames, n, world, device=None):
    """Whole-job figures of one timed region of ``n`` steps: (ms per step, frames per step summed over
    the ranks). The time is the slowest rank's (all_reduce MAX), the frames the sum (all_reduce SUM);
    weak scaling. ``device``: where the reduction tensors live (the rank's GPU under nccl, the CPU
    under gloo)."""
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([frames / n], device=device, dtype=torch.float64)
        m = torch.tensor([el_s], device=device, dtype=torch.float64)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        el_s, per = float(m.item()), int(round(t.item()))
    else:
        per = frames // n
    return el_s / n * 1000.0, per


def bench_config(world, per_gpu_batch, r):
    """The line's ``config``: C2 at one GPU, C3 (replicas, weak scaling) above."""
    return {"workload": f"C{2 if world == 1 else 3}: Tacotron2-DDC (r_init=7, r={r}, sigmoid attn) + "
                        f"MB-MelGAN [8,4,2]x4, {per_gpu_batch} LJ-length utterances per GPU",
            "global_batch": per_gpu_batch * world, "r": r, "parallelism": f"replicas x{world}"}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


def launch_plan(gpus, env, argv):
    """What ``python bench.py --gpus N`` must do before anything touches a GPU (one process per GPU,
    as TTS/bin/distribute.py:41-65 starts one training process per GPU):
    * no WORLD_SIZE and N > 1: start N ranks under torch.distributed.run as a CHILD process (never
      exec) with the same arguments, and exit with its return code -> returns that command;
    * WORLD_SIZE set (already a rank of a launcher) and equal to N, or N == 1 with no WORLD_SIZE:
      run in this process -> returns None;
    * WORLD_SIZE set and different from N: refused (SystemExit with a message, status 2)."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}; launch N ranks with "
                             f"--gpus N (or drop --gpus and let bench.py start them)")
        return None
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    if gpus == 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(env.get("MASTER_PORT") or free_port()),
            os.path.abspath(__file__)] + list(argv)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--r", type=int, default=2)
    ap.add_argument("--per-gpu-batch", type=int, default=32)
    ap.add_argument("--cpu-seconds", type=float, default=30.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--f32-steps", type=int, default=3, help="steps re-timed with fp32-MFMA GEMMs only (0: skip)")
    ap.add_argument("--r1-steps", type=int, default=3, help="steps timed at r=1 as extra fields (0: skip)")
    ap.add_argument("--plan-only", action="store_true",
                    help="print this rank's shard of the global batch as one JSON line and exit (no GPU)")
    args = ap.parse_args(argv)

    # before any torch.cuda call (not even device_count): become the launcher of N ranks if asked
    cmd = launch_plan(args.gpus, os.environ, argv)
    if cmd is not None:
        import subprocess
        return subprocess.call(cmd)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plan_only:
        mine, my_T, _, _ = rank_shard(world, rank, args.per_gpu_batch, args.r)
        print(json.dumps({"rank": rank, "world": world, "local_rank": local, "shard": [int(i) for i in mine],
                          "tokens": [int(t_) for t_ in my_T]}), flush=True)
        return 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    taco, tsd, voc, vsd, tcfg, vcfg = build_models(dev)
    taco.decoder.verbose = False  # forced lengths end every utterance at max_decoder_steps
    # the rank's share of the global batch (rank_shard: tts_amd.multigpu's LPT plan)
    mine, my_T, my_prof, M_all = rank_shard(world, rank, args.per_gpu_batch, args.r)
    T_prof, M_prof = lj_profile()
    ids = synthetic_ids(T_prof)              # C3 replicates the same 32 utterances
    my_ids = [ids[i] for i in my_prof]
    batch, lens = pad_batch(my_ids)
    batch_t = torch.from_numpy(batch).to(dev)
    batch_host = torch.from_numpy(batch).pin_memory()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tt, tv = [], []

    def one_step(steps, record=False, two_calls=False):
        """One batch through both models. Default: ONE library call (Tacotron2.inference_vocoded ->
        tts_taco_mbmelgan_infer, the decoded lengths handed to the vocoder inside the library).
        ``two_calls`` / ``record``: the reference's call pattern, Tacotron2.inference then
        MultibandMelganGenerator.inference (the stage split is event-timed on that form)."""
        if not (record or two_calls):
            wav = taco.inference_vocoded(batch_t, voc, text_lengths=lens, max_decoder_steps=steps)[4]
            return int(taco.last_mel_lengths.sum()), wav
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

    wav_host = {}

    def host_step(steps):
        """IDs on the host -> waveforms on the host (SURVEY 8d e2e RTF; server/synthesizer.py:147,155-156):
        H2D of the pinned id batch, both models, D2H of the waveform batch into pinned memory and the
        per-utterance cut to its own 256 * M_i samples."""
        x = batch_host.to(dev, non_blocking=True)
        wav = taco.inference_vocoded(x, voc, text_lengths=lens, max_decoder_steps=steps)[4]
        mel_lens = taco.last_mel_lengths
        key = tuple(wav.shape)
        if key not in wav_host:
            wav_host[key] = torch.empty(key, dtype=wav.dtype, pin_memory=True)
        h = wav_host[key]
        h.copy_(wav, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        hn = h.numpy()
        return [hn[i, 0, :HOP * int(m)] for i, m in enumerate(mel_lens)]

    def pipelined(steps, n):
        """n batches through both models with the host one batch ahead (Tacotron2.
        inference_vocoded_submit -> tts_taco_mbmelgan_submit / _finish): batch i + 1 is submitted,
        its encoder and decode running beside batch i's vocoder (the library's second stream), before
        batch i's result is taken.
        Every batch's waveforms are final (range flag checked) inside the caller's timed region."""
        frames = 0
        prev = None
        for _ in range(n):
            cur = taco.inference_vocoded_submit(batch_t, voc, text_lengths=lens, max_decoder_steps=steps)
            frames += int(taco.last_mel_lengths.sum())
            if prev is not None:
                prev.result()
            prev = cur
        if prev is not None:
            prev.result()
        return frames

    def timed_pipelined(steps, n):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        frames = pipelined(steps, n)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return aggregate(time.perf_counter() - t0, frames, n, world, dev)

    def timed(fn, n):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        frames = 0
        for _ in range(n):
            out = fn()
            frames += out[0] if isinstance(out, tuple) else sum(len(w) for w in out) // HOP
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return aggregate(time.perf_counter() - t0, frames, n, world, dev)

    from tts_amd._lib import get_engine
    eng = get_engine(dev)

    def measure(r, steps_n, warmup, with_host):
        """One configuration (reduction factor r): the timed device-resident step, the stage split,
        the host-to-host step, and the decoder launch statistics."""
        taco.decoder.set_r(r)
        steps = forced_steps([M_all[i] for i in mine], r)
        for _ in range(warmup):
            one_step(steps)
        pipelined(steps, 2)
        ms, per_frames = timed_pipelined(steps, steps_n)
        sync_ms, _ = timed(lambda: one_step(steps), steps_n)  # one synchronous fused call per batch
        two_ms, _ = timed(lambda: one_step(steps, two_calls=True), steps_n)  # the reference's two-call form
        tt.clear()
        tv.clear()
        for _ in range(2):  # per-stage split (separate, event-timed passes after the timed region)
            one_step(steps, True)
        path, launches = eng.decoder_stats()
        res = {"ms": ms, "sync_ms": sync_ms, "two_call_ms": two_ms, "frames": per_frames, "steps": steps, "taco_ms": float(np.median(tt)),
               "voc_ms": float(np.median(tv)), "path": path, "launches": launches}
        if with_host:
            host_step(steps)
            res["host_ms"], _ = timed(lambda: host_step(steps), steps_n)
        bound, dec_bound = pipeline_bound_ms(my_T, steps, r)
        bound_x3, _ = pipeline_bound_ms(my_T, steps, r, X3_PEAK_TFLOPS)
        res.update(bound_ms=bound, dec_bound_ms=dec_bound, bound_x3_ms=bound_x3)
        return res

    r = args.r
    m2 = measure(r, args.steps, args.warmup, with_host=True)
    ms_step, per_step_frames, steps = m2["ms"], m2["frames"], m2["steps"]
    value = per_step_frames / (ms_step / 1000.0)
    audio_s = per_step_frames * HOP / SAMPLE_RATE
    taco_ms, voc_ms = m2["taco_ms"], m2["voc_ms"]
    my_frames = int(sum(s_ * r for s_ in steps))
    gemm_mode, fallbacks = eng.gemm_mode()
    path, launches = m2["path"], m2["launches"]

    # the same step with every GEMM on the fp32 MFMA (no split-f16 kernels), for comparison
    f32_ms = None
    if gemm_mode == "x3" and args.f32_steps > 0:
        eng.set_gemm_mode("f32")
        try:
            one_step(steps)
            f32_ms, _ = timed_pipelined(steps, args.f32_steps)
        finally:
            eng.set_gemm_mode("x3")

    # the other reduction factor SURVEY 8d asks for (r=1: 858 decoder steps), as extra fields
    other = None
    if args.r1_steps > 0 and r == 2:
        m1 = measure(1, args.r1_steps, 1, with_host=False)
        _, st1 = m1["launches"][0]
        other = {"r": 1, "ms_per_step": round(m1["ms"], 3), "mel_frames_per_s": round(m1["frames"] / (m1["ms"] / 1e3), 1),
                 "e2e_rtf": m1["ms"] / 1000.0 / (m1["frames"] * HOP / SAMPLE_RATE),
                 "tacotron2_mel_frames_per_s": round(sum(m1["steps"]) / (m1["taco_ms"] / 1e3) * world, 1),
                 "tacotron2_ms": round(m1["taco_ms"], 3), "vocoder_ms": round(m1["voc_ms"], 3),
                 "decoder_steps": int(max(m1["steps"])),
                 "decoder_step_us": round(m1["launches"][0][0] / max(st1, 1) * 1000.0, 2) if m1["path"] == 1 else None,
                 "pipeline_bound_ms": round(m1["bound_ms"], 3), "pipeline_frac": round(m1["bound_ms"] / m1["ms"], 4),
                 "pipeline_frac_x3_ceiling": round(m1["bound_x3_ms"] / m1["ms"], 4)}
        taco.decoder.set_r(r)

    # dominant decoder kernel, timed live with HIP events on the library's stream (stats above)
    if path == 1:
        # persistent decoder: the MT = 2 launch (32-row batch tile) carries most steps. Algorithmic
        # work = useful row-steps (rows still decoding) x the per-row GEMM flops of one step, plus
        # the attention's 13,440 FLOP per (row, step, encoder position)
        ms0, st0 = launches[0]
        flop_row = 2 * (4096 * 2560          # decoder_rnn [W_ih | W_hh]
                        + 4096 * 1536        # attention_rnn ctx/h part
                        + 4096 * 256         # attention_rnn prenet part
                        + (1 + 80 * r) * 1536  # projection (r frames) + stopnet
                        + 80 * 256 + 256 * 256  # prenet
                        + 1024 * 128)        # query projection
        rows = range(min(len(mine), 16 * ((len(mine) + 15) // 16)))
        row_steps = sum(min(steps[i], st0) for i in rows)
        att_flops = sum(ATT_FLOP_PER_T * my_T[i] * min(steps[i], st0) for i in rows)
        flops = row_steps * flop_row + att_flops
        achieved = flops / (ms0 * 1e-3) / 1e12
        # SURVEY 8d's named bound for the decoder: HBM. Algorithmic bytes of the launch = per step the
        # decoder weights (75.71 MB, read once per batched step in the reference's op sequence) + per
        # active row 2,580 T (inputs, processed inputs, alpha / alpha_cum, alignment write) + 320 r
        # (frames) + ~37.5 KB (states): the figures pipeline_bound_ms uses
        alg_bytes = st0 * DEC_W_BYTES + sum(min(steps[i], st0) * (2580.0 * my_T[i] + 320.0 * r + 37_500.0) for i in rows)
        achieved_gbs = alg_bytes / (ms0 * 1e-3) / 1e9
        step_ms = ms0 / max(st0, 1)
        traffic, traffic_src = None, None
        pmc = latest_profile("persist_pmc.json")
        if pmc:
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
                traffic_src = os.path.relpath(pmc, ROOT)
            except Exception:
                traffic = None
        # split-f16 mode: the decoder's GEMM parts run 3 f16 MFMAs per fp32 product, so the
        # ceiling is the f16 MFMA peak / 3 in fp32-equivalent FLOP/s; fp32 mode: the fp32 MFMA peak
        peak = X3_PEAK_TFLOPS if gemm_mode == "x3" else F32_PEAK_TFLOPS
        # what the step actually hits is the latency of its hand-off chain (5 phases per step, each
        # separated by a grid barrier, each starting with a coherent load of what the previous one
        # published): tools/chain_bench.hip runs that chain with the decoder's roles and hand-off
        # sizes and no arithmetic (the newest profiles/rNN/chain_floor.json; round 5 re-ran it with the
        # flag barrier the kernel now uses). achieved / peak stay the MFMA
        # figures (algorithmic FLOPs / launch time against the split-f16 ceiling)
        floor = None
        fpath = latest_profile("chain_floor.json")
        if fpath:
            try:
                floor = json.load(open(fpath))
            except Exception:
                floor = None
        # bound / achieved / peak / frac: SURVEY 8d's HBM roofline on the algorithmic bytes (the
        # kernel keeps the weights on chip, so traffic, the PMC-counted HBM bytes per launch, is far
        # below them); mfma_*: the same launch against the MFMA ceiling of its arithmetic; the step
        # itself is latency-bound (latency_floor_*: the hand-off chain without arithmetic)
        roof = {"kernel": "persist_decoder_kernel<2%s> (whole decoder loop, weights resident on chip)"
                          % (", split-f16" if gemm_mode == "x3" else ""),
                "bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes": int(alg_bytes),
                "traffic": traffic, "traffic_source": traffic_src,
                "regime": "latency (5 grid barriers and hand-off round trips per step; see latency_floor_*)",
                "mfma_achieved_tflops": round(achieved, 2), "mfma_peak_tflops": peak,
                "mfma_frac": round(achieved / peak, 4), "mfma_frac_vs_fp32_peak": round(achieved / F32_PEAK_TFLOPS, 4),
                "algorithmic_flops": flops,
                "avg_launch_us": round(ms0 * 1000.0, 1), "launch_steps": st0,
                "launches": [[round(m_, 3), s_] for m_, s_ in launches]}
        if floor:
            fl = floor["loads_barriers_us"]
            roof.update({"step_us": round(step_ms * 1000.0, 2),
                         "latency_floor_us": fl,
                         "latency_floor_barriers_only_us": floor["noload_barriers_us"],
                         "latency_floor_with_compute_standins_us": floor["compute_loads_barriers_us"],
                         "frac_of_latency_floor": round(fl / (step_ms * 1000.0), 4),
                         "latency_floor_source": os.path.relpath(fpath, ROOT) + ": 5 grid barriers + the phases' "
                                                 "coherent hand-off loads per step, no arithmetic"})
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
    # SURVEY 8d whole-pipeline bound (fp32 peaks) / measured, and the same with the compute part
    # priced at the split-f16 ceiling the kernels actually run at
    roof["pipeline_bound_ms"] = round(m2["bound_ms"], 3)
    roof["pipeline_frac"] = round(m2["bound_ms"] / ms_step, 4)
    roof["pipeline_frac_x3_ceiling"] = round(m2["bound_x3_ms"] / ms_step, 4)
    roof["decoder_bound_ms"] = round(m2["dec_bound_ms"], 3)
    if path == 1:
        dec_ms = sum(m_ for m_, _ in launches)
        roof["decoder_frac"] = round(m2["dec_bound_ms"] / dec_ms, 4)

    host_audio = per_step_frames * HOP / SAMPLE_RATE
    out = {
        "metric": "mel-frames/s (Tacotron2-DDC + MB-MelGAN end-to-end)",
        "value": round(value, 1),
        "unit": "mel-frames/s",
        "n_gpus": world,
        "rccl_world": dist.get_world_size() if world > 1 else 1,
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
        "config": bench_config(world, args.per_gpu_batch, r),
        "e2e_rtf": ms_step / 1000.0 / audio_s,
        "e2e_rtf_host": m2["host_ms"] / 1000.0 / host_audio,
        "host_ms_per_step": round(m2["host_ms"], 3),
        "sync_call_ms_per_step": round(m2["sync_ms"], 3),
        "two_call_ms_per_step": round(m2["two_call_ms"], 3),
        "entry": "Tacotron2.inference_vocoded_submit -> tts_taco_mbmelgan_submit / _finish, the host one batch "
                 "ahead (batch i+1's Tacotron2 beside batch i's vocoder on the library's second stream); sync_call_ms_per_step: one blocking "
                 "tts_taco_mbmelgan_infer per batch; two_call_ms_per_step: Tacotron2.inference + "
                 "MultibandMelganGenerator.inference",
        "tacotron2_mel_frames_per_s": round(my_frames / (taco_ms / 1000.0) * world, 1),
        "tacotron2_ms": round(taco_ms, 3),
        "vocoder_ms": round(voc_ms, 3),
        "decoder_step_us": round(step_ms * 1000.0, 2),
        "decoder_steps": int(max(steps)),
        "decoder_path": "persistent" if path == 1 else "step-graphs",
        "roofline": roof,
        "r1": other,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(tsd, vsd, tcfg, vcfg, ids, forced_steps(M_prof, r), r,
                                           args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
