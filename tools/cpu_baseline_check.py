"""Times the imported REFERENCE CPU path beside the numpy oracle (bench.py's cpu_baseline leg) in
THIS container, on the same weights, LJ-profile utterances and forced lengths, so the
oracle's host-CPU number on the GPU box can be read against the reference's. Build container only
(the reference never travels to the GPU box):

    PYTHONPATH=/root/reference:/root/repo python tools/cpu_baseline_check.py [--threads 8] [--r 2]

Writes profiles/<round>/cpu_baseline_check_r{r}.json (--round, default r05).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = os.environ.get("TTS_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

from tts_amd.spec import MelganConfig, TacotronConfig, melgan_layers, melgan_spec, tacotron2_spec  # noqa: E402
from tts_amd.weights import synth_state_dict  # noqa: E402
from tts_amd.workload import HOP, SAMPLE_RATE, forced_steps, lj_profile, synthetic_ids  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--r", type=int, default=2)
    ap.add_argument("--n", type=int, default=32, help="utterances (file order)")
    ap.add_argument("--round", default="r05", help="profiles/ subdirectory the record goes to")
    args = ap.parse_args()
    from threadpoolctl import threadpool_limits
    from TTS.tts.models.tacotron2 import Tacotron2
    from TTS.vocoder.models.multiband_melgan_generator import MultibandMelganGenerator
    from oracle.melgan_np import MelganOracle
    from oracle.taco_np import TacoOracle
    from oracle.torch_cpu import MelganTorchCPU, TacoTorchCPU
    from tts_amd.pqmf import pqmf_filters

    torch.set_num_threads(args.threads)
    r = args.r
    tcfg, vcfg = TacotronConfig(), MelganConfig()
    tsd = synth_state_dict(tacotron2_spec(tcfg), 0)          # bench.py's weights (seed 0 / 1)
    tsd["decoder.stopnet.1.linear_layer.bias"] = np.array([-1e4], np.float32)
    vsd = synth_state_dict(melgan_spec(vcfg, weight_norm=True), 1)
    T_prof, M_prof = lj_profile()
    ids = synthetic_ids(T_prof)[:args.n]
    steps = forced_steps(M_prof, r)[:args.n]

    taco = Tacotron2(num_chars=tcfg.num_chars, num_speakers=0, r=tcfg.r, attn_norm=tcfg.attn_norm,
                     double_decoder_consistency=True, ddc_r=tcfg.ddc_r)
    full = taco.state_dict()
    for k, v in tsd.items():
        full[k] = torch.from_numpy(np.asarray(v))
    taco.load_state_dict(full)
    taco.eval()
    taco.decoder.set_r(r)
    voc = MultibandMelganGenerator(in_channels=80, out_channels=4, base_channels=384,
                                   upsample_factors=list(vcfg.upsample_factors), num_res_blocks=vcfg.num_res_blocks)
    full = voc.state_dict()
    for k, v in vsd.items():
        full[k] = torch.from_numpy(v)
    voc.load_state_dict(full)
    voc.remove_weight_norm()
    voc.inference_padding = 0
    voc.eval()

    def ref_one(i):
        taco.decoder.max_decoder_steps = int(steps[i])
        with torch.no_grad():
            t0 = time.perf_counter()
            _, post, _, _ = taco.inference(torch.from_numpy(ids[i][None].astype(np.int64)))
            t1 = time.perf_counter()
            voc.inference(post.transpose(1, 2))
            t2 = time.perf_counter()
        return post.shape[1], t1 - t0, t2 - t1, post[0].numpy()

    to = TacoOracle(tsd, tcfg.attn_norm, tcfg.r)
    vo = MelganOracle(vsd, melgan_layers(vcfg), pqmf_filters()[1])

    def orc_one(i):
        t0 = time.perf_counter()
        _, p, _, _ = to.inference(ids[i], r, int(steps[i]))
        t1 = time.perf_counter()
        vo.inference(p.T, pad=0)
        t2 = time.perf_counter()
        return p.shape[0], t1 - t0, t2 - t1, p

    ta = TacoTorchCPU(tsd, tcfg.attn_norm, tcfg.r)
    va = MelganTorchCPU(vsd, melgan_layers(vcfg), pqmf_filters()[1])

    def aten_one(i):
        t0 = time.perf_counter()
        _, p, _, _ = ta.inference(ids[i], r, int(steps[i]))
        t1 = time.perf_counter()
        va.inference(p.T, pad=0)
        t2 = time.perf_counter()
        return p.shape[0], t1 - t0, t2 - t1, p

    res = {}
    j = int(np.argmin(steps))
    with threadpool_limits(limits=args.threads):
        for name, fn in (("reference", ref_one), ("aten_port", aten_one), ("oracle", orc_one)):
            fn(j)  # warm-up, excluded
            frames, tt, tv = 0, 0.0, 0.0
            posts = []
            for i in range(len(ids)):
                f, a, b, p = fn(i)
                frames += f
                tt += a
                tv += b
                posts.append(p)
            audio = frames * HOP / SAMPLE_RATE
            res[name] = {"frames": frames, "tacotron2_s": round(tt, 3), "vocoder_s": round(tv, 3),
                         "tacotron2_frames_per_s": round(frames / tt, 1), "e2e_frames_per_s": round(frames / (tt + tv), 1),
                         "e2e_rtf": round((tt + tv) / audio, 5)}
            res[name + "_posts"] = posts
            print(name, res[name], flush=True)
    refp = res.pop("reference_posts")
    err = max(float(np.abs(a - b).max()) for a, b in zip(refp, res.pop("oracle_posts")))
    err_a = max(float(np.abs(a - b).max()) for a, b in zip(refp, res.pop("aten_port_posts")))
    out = {"r": r, "threads": args.threads, "utterances": len(ids), "torch": torch.__version__,
           "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
           "oracle_vs_reference_post_max_abs": err, "aten_port_vs_reference_post_max_abs": err_a, **res,
           "aten_port_over_reference_tacotron2": round(res["aten_port"]["tacotron2_frames_per_s"]
                                                       / res["reference"]["tacotron2_frames_per_s"], 3),
           "aten_port_over_reference_e2e": round(res["aten_port"]["e2e_frames_per_s"]
                                                 / res["reference"]["e2e_frames_per_s"], 3),
           "oracle_over_reference_tacotron2": round(res["oracle"]["tacotron2_frames_per_s"]
                                                    / res["reference"]["tacotron2_frames_per_s"], 3),
           "oracle_over_reference_e2e": round(res["oracle"]["e2e_frames_per_s"] / res["reference"]["e2e_frames_per_s"], 3)}
    path = os.path.join(ROOT, "profiles", args.round, f"cpu_baseline_check_r{r}.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
