"""ORACLE (test infrastructure only): float32 numpy restatement of the reference
MultiBand-MelGAN generator + PQMF synthesis. Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.

Parity pin: ``tests/golden/mbmelgan.npz`` and ``tests/golden/pqmf.npz`` (reference outputs,
``tests/golden/make_golden.py``) plus the reference's own known answer
``TTS/vocoder/pqmf_output.wav`` (stored in ``pqmf.npz``).

Reference op sequences (paths relative to the reference checkout):

* ``TTS/vocoder/models/melgan_generator.py:28-78``  layer stack
* ``TTS/vocoder/models/melgan_generator.py:91-97`` + ``TTS/vocoder/layers/melgan.py:41-45``
  remove_weight_norm: w = g * v / ||v|| (norm over every dim but 0)
* ``TTS/vocoder/layers/melgan.py:35-39``  ResidualStack: x = shortcut(x) + block(x)
* ``TTS/vocoder/models/multiband_melgan_generator.py:32-39``  inference (replicate pad)
* ``TTS/vocoder/layers/pqmf.py:51-56``  synthesis = conv_transpose1d(updown*N, stride N)
  then conv1d(G, padding taps//2)
"""

import numpy as np

from oracle.taco_np import conv1d

F32 = np.float32


def wn_fold(g, v):
    """weight_norm dim=0: w = g * v / ||v||_2 over all dims except 0."""
    v = v.astype(F32)
    n = np.sqrt((v.astype(np.float64) ** 2).reshape(v.shape[0], -1).sum(1)).astype(F32)
    return (v * (g.reshape(-1) / n).reshape((-1,) + (1,) * (v.ndim - 1))).astype(F32)


def reflect_pad(x, p):
    if p == 0:
        return x
    L = x.shape[1]
    if p >= L:
        raise RuntimeError("ReflectionPad1d: padding must be < input length")
    left = x[:, p:0:-1]
    right = x[:, L - 2:L - 2 - p:-1]
    return np.concatenate([left, x, right], axis=1)


def leaky_relu(x, s=0.2):
    return np.where(x >= 0, x, x * F32(s)).astype(F32)


def conv_transpose1d(x, w, b, stride, padding, output_padding=0):
    """torch ConvTranspose1d; x (Cin, L), w (Cin, Cout, K)."""
    cin, L = x.shape
    _, cout, K = w.shape
    Lfull = (L - 1) * stride + K + output_padding
    cols = (w.reshape(cin, cout * K).T.astype(F32) @ x).reshape(cout, K, L)
    y = np.zeros((cout, Lfull), F32)
    for k in range(K):
        y[:, k:k + stride * (L - 1) + 1:stride] += cols[:, k, :]
    y = y[:, padding:Lfull - padding]
    if b is not None:
        y = y + b[:, None]
    return y.astype(F32)


class MelganOracle:
    def __init__(self, sd, layers, pqmf_G=None):
        """``sd``: state_dict (weight_g/weight_v or folded weight); ``layers``: spec list
        from ``tts_amd.spec.melgan_layers``."""
        self.layers = layers
        self.w, self.b = {}, {}
        for l in layers:
            if f"{l.name}.weight" in sd:
                w = np.asarray(sd[f"{l.name}.weight"], F32)
            else:
                w = wn_fold(np.asarray(sd[f"{l.name}.weight_g"], F32), np.asarray(sd[f"{l.name}.weight_v"], F32))
            self.w[l.name] = w
            self.b[l.name] = np.asarray(sd[f"{l.name}.bias"], F32)
        self.G = None if pqmf_G is None else np.asarray(pqmf_G, F32)

    def generator(self, c):
        """self.layers(c) for one utterance, c (80, L) -> (4, 256/4 * L)."""
        ls = self.layers
        x = conv1d(reflect_pad(c.astype(F32), ls[0].padding), self.w[ls[0].name], self.b[ls[0].name])
        i = 1
        while i < len(ls) and ls[i].kind == "convT":
            l = ls[i]
            x = conv_transpose1d(leaky_relu(x), self.w[l.name], self.b[l.name], l.stride, l.padding,
                                 l.extra.get("output_padding", 0))
            i += 1
            while i < len(ls) and ls[i].kind == "res_dconv":
                dc, pw, sc = ls[i], ls[i + 1], ls[i + 2]
                h = leaky_relu(x)
                h = conv1d(reflect_pad(h, dc.padding), self.w[dc.name], self.b[dc.name],
                           dilation=dc.dilation)
                h = conv1d(leaky_relu(h), self.w[pw.name], self.b[pw.name])
                x = (conv1d(x, self.w[sc.name], self.b[sc.name]) + h).astype(F32)
                i += 3
        l = ls[i]
        x = conv1d(reflect_pad(leaky_relu(x), l.padding), self.w[l.name], self.b[l.name])
        return np.tanh(x).astype(F32)

    def pqmf_synthesis(self, x):
        return pqmf_synthesis(x, self.G)

    def inference(self, c, pad=2):
        """MultibandMelganGenerator.inference for one utterance, c (80, M)."""
        c = np.asarray(c, F32)
        if pad:
            c = np.concatenate([np.repeat(c[:, :1], pad, 1), c, np.repeat(c[:, -1:], pad, 1)], 1)
        return self.pqmf_synthesis(self.generator(c))


def pqmf_synthesis(x, G):
    """PQMF.synthesis (pqmf.py:51-56): x (N, L) -> (1, N*L)."""
    N, L = x.shape
    taps = G.shape[-1] - 1
    u = np.zeros((N, N * L), F32)
    u[:, ::N] = x * F32(N)
    return conv1d(u, G.reshape(1, N, taps + 1), None, padding=taps // 2)
