"""Multi-GPU Synthesizer check on a GPU box: Synthesizer(config with gpu_devices) shards a call's
sentences over one worker process per listed device (tts_amd.multigpu.GpuPool; a one-GPU box lists
device 0 twice), and every sentence's waveform must match the oracle chain (TacoOracle ->
MelganOracle) at B = 1. This process never touches the GPU itself (the workers do), so it is run as
a fresh child process: tests/test_gpu_parity.py::test_synthesizer_gpu_pool_vs_oracle_chain.

    python tools/pool_check.py <scratch dir> [devices, e.g. 0,0]
"""
import os
import pathlib
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(argv):
    tmp = pathlib.Path(argv[0])
    devices = [int(d) for d in (argv[1] if len(argv) > 1 else "0,0").split(",")]
    import test_gpu_parity as T
    from oracle.taco_np import TacoOracle
    from helpers import melgan_oracle
    from tts_amd.synthesizer import Synthesizer
    from tts_amd.text import text_to_seqvec

    conf = T._synth_files(tmp, stats=True)
    conf["gpu_devices"] = devices
    conf["max_decoder_steps"] = 24  # the stop bias of these weights never fires: every sentence decodes 24 steps
    synth = Synthesizer(conf)
    try:
        assert synth.pool is not None and len(synth.pool.devices) == len(devices)
        assert synth.tts_model is None and synth.vocoder_model is None  # the models live in the workers
        cfg, sd, mcfg, msd = T._synth_models()
        to, vo = TacoOracle(sd, cfg.attn_norm, cfg.r), melgan_oracle(mcfg, msd)
        sens = ["Hello world.", "This is a longer test of the sharded path, with 2 numbers!", "Short one?",
                "A fourth sentence goes to whichever worker is lighter."]
        wavs = synth.synthesize_batch(sens)
        assert len(wavs) == len(sens)
        worst = 0.0
        for s_, w in zip(sens, wavs):
            ids = text_to_seqvec(s_, synth.tts_config)
            _, p, _, _ = to.inference(ids, 2, 24)
            ref = vo.inference(p.T, pad=0).reshape(-1)
            assert w.shape == ref.shape, (s_, w.shape, ref.shape)
            err = float(np.abs(w - ref).max())
            worst = max(worst, err)
            assert err <= 1e-4, (s_, err)
        buf = synth.tts(" ".join(sens))
        assert len(buf.getvalue()) > 44
    finally:
        synth.close()
    print(f"pool ok: {len(sens)} sentences over devices {devices}, worst waveform error {worst:.2e}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
