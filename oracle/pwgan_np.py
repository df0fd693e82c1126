"""ORACLE (test infrastructure only): float32 numpy restatement of ParallelWaveGAN generator
inference. Only ``tests/`` may import it.

Parity pin: ``tests/golden/pwgan.npz`` was produced in the build container by the reference's own
``ParallelWaveganGenerator.inference`` with the prior noise captured by re-seeding torch (see
make_golden.py ``pwgan``).

* ``vocoder/models/parallel_wavegan_generator.py:90-125``  replicate pad, noise, upsample,
  first_conv, residual blocks, skip sum * sqrt(1 / layers), ReLU-conv-ReLU-conv
* ``vocoder/layers/upsample.py:5-101``  ConvUpsample: conv_in (1x1), per factor s nearest stretch
  then a (1, 2s + 1) Conv2d with zero padding s shared by all channels
* ``vocoder/layers/parallel_wavegan.py:56-87``  dilated conv + 1x1 aux, tanh * sigmoid gate,
  skip / out 1x1, (out + residual) * 0.25
"""

import math

import numpy as np

F32 = np.float32


def fold_weight_norm(sd):
    """w = g * v / ||v|| over all but dim 0 (torch.nn.utils.weight_norm, dim 0)."""
    out = {}
    for k, v in sd.items():
        if k.endswith(".weight_v"):
            base = k[:-len(".weight_v")]
            g = sd[base + ".weight_g"].astype(np.float64)
            vv = v.astype(np.float64)
            n = np.sqrt((vv.reshape(vv.shape[0], -1) ** 2).sum(1)).reshape((-1,) + (1,) * (vv.ndim - 1))
            out[base + ".weight"] = (vv / n * g).astype(F32)
        elif not k.endswith(".weight_g"):
            out[k] = v
    return out


def dconv(x, w, b, d):
    """x (Cin, L), w (Cout, Cin, K) dilated by d, zero padding (K - 1) / 2 * d (same length)."""
    cout, cin, K = w.shape
    p = (K - 1) // 2 * d
    L = x.shape[1]
    xp = np.pad(x, ((0, 0), (p, p)))
    y = np.zeros((cout, L), F32)
    for k in range(K):  # contiguous tap slice: a strided one makes numpy skip BLAS (~100x slower)
        y += np.ascontiguousarray(w[:, :, k]) @ xp[:, k * d:k * d + L]
    if b is not None:
        y += b[:, None]
    return y.astype(F32)


class PwganOracle:
    def __init__(self, sd, cfg):
        self.w = fold_weight_norm(sd)
        self.c = cfg

    def upsample(self, c):
        w = self.w
        c = dconv(c, w["upsample_net.conv_in.weight"], None, 1)
        for i, s in enumerate(self.c.upsample_factors):
            h = w[f"upsample_net.upsample.up_layers.{2 * i + 1}.weight"].reshape(-1)
            u = np.repeat(c, s, axis=1)
            L = u.shape[1]
            up = np.pad(u, ((0, 0), (s, s)))
            c = np.zeros_like(u)
            for k in range(2 * s + 1):
                c += h[k] * up[:, k:k + L]
            c = c.astype(F32)
        return c

    def inference(self, mel, noise):
        """mel (80, M), noise (T,) with T = (M + 2 pad) * 256 -> waveform (T,)."""
        w, cfg = self.w, self.c
        p = cfg.inference_padding
        c = np.pad(mel, ((0, 0), (p, p)), mode="edge").astype(F32)
        c = self.upsample(c)
        x = (w["first_conv.weight"].reshape(-1, 1) * noise[None, :] + w["first_conv.bias"][:, None]).astype(F32)
        skips = np.zeros((cfg.skip_channels, x.shape[1]), F32)
        H = cfg.gate_channels // 2
        for i in range(cfg.num_res_blocks):
            q = f"conv_layers.{i}."
            a = dconv(x, w[q + "conv.weight"], w[q + "conv.bias"], cfg.dilation(i))
            a = a + w[q + "conv1x1_aux.weight"][:, :, 0] @ c
            z = (np.tanh(a[:H]) * (1.0 / (1.0 + np.exp(-a[H:])))).astype(F32)
            s = w[q + "conv1x1_skip.weight"][:, :, 0] @ z + w[q + "conv1x1_skip.bias"][:, None]
            x = ((w[q + "conv1x1_out.weight"][:, :, 0] @ z + w[q + "conv1x1_out.bias"][:, None] + x) * F32(0.25))
            x = x.astype(F32)
            skips = (skips + s).astype(F32)
        skips = skips * F32(math.sqrt(1.0 / cfg.num_res_blocks))
        h = np.maximum(skips, 0)
        h = np.maximum(w["last_conv_layers.1.weight"][:, :, 0] @ h + w["last_conv_layers.1.bias"][:, None], 0)
        y = w["last_conv_layers.3.weight"][:, :, 0] @ h + w["last_conv_layers.3.bias"][:, None]
        return y[0].astype(F32)
