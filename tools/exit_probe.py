"""Exit-path probe under rocprofv3 (bisects a crash in process teardown).

stage 0: torch only; 1: + library context; 2: + Tacotron2 inference; 3: + MB-MelGAN inference.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

stage = int(sys.argv[1])
dev = torch.device("cuda:0")
torch.zeros(1, device=dev).add_(1)
torch.cuda.synchronize()
if stage >= 1:
    from tts_amd import _lib
    _lib.get_engine(dev)
if stage >= 2:
    from helpers import build_melgan, build_taco, melgan_state_dict, taco_state_dict
    from tts_amd.spec import TacotronConfig
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=1, overrides={}, stop_bias=-1e4, cfg=cfg)
    m = build_taco(cfg, sd, dev)
    m.decoder.set_r(2)
    ids = np.random.RandomState(0).randint(1, 129, size=(1, 21)).astype(np.int64)
    dec, post, align, stop = m.inference(torch.from_numpy(ids).to(dev), max_decoder_steps=6)
if stage >= 3:
    vcfg, vsd = melgan_state_dict(3)
    v = build_melgan(vcfg, vsd, dev)
    v.inference(post.transpose(1, 2).contiguous())
torch.cuda.synchronize()
print("stage", stage, "done", flush=True)
if len(sys.argv) > 2:  # library map, to resolve the addresses of a teardown crash
    with open("/proc/self/maps") as f, open(sys.argv[2], "w") as g:
        g.write(f.read())
