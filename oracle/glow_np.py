"""ORACLE (test infrastructure only): float32 numpy restatement of Glow-TTS inference for the
reference configs (gated-conv encoder, mean_only, num_sqz 2, num_splits 4, dilation 1). Only
``tests/`` may import it.

Parity pin: ``tests/golden/glow.npz`` was produced in the build container by the reference's own
``Encoder`` / ``Decoder`` modules (``TTS/tts/layers/glow_tts/{encoder,decoder}.py``) composed with
the inference glue of ``TTS/tts/models/glow_tts.py:166-193`` (that module itself does not import
here: its ``monotonic_align.core`` Cython extension is not built), see make_golden.py ``glow``.

* ``layers/glow_tts/encoder.py:105-130``  embedding * sqrt(H), GatedConvBlock / ConvLayerNorm prenet +
  TimeDepthSeparableConvBlock / Transformer (``transformer.py:9-127,228-319``), proj_m, durations
* ``layers/glow_tts/gated_conv.py:31-42``  conv -> LayerNorm -> GLU -> residual
* ``layers/glow_tts/normalization.py:4-27,77-89``  LayerNorm (eps 1e-4), ActNorm reverse
* ``layers/glow_tts/duration_predictor.py:29-40``
* ``models/glow_tts.py:170-193``  w_ceil, y_lengths, generate_path, expanded means, noise
* ``layers/glow_tts/decoder.py:6-33,81-95``  squeeze / unsqueeze, flows reversed
* ``layers/glow_tts/glow.py:85-138,171-205,245-262``  WN, InvConvNear reverse, CouplingBlock reverse
* speaker conditioning: ``models/glow_tts.py:159-161`` g = F.normalize(emb_g(speaker)),
  ``encoder.py:131-135`` [x; g] into the duration predictor, ``glow.py:119-130`` cond_layer(g) sliced
  per WN layer and added before the gate (pinned by ``tests/golden/glow_spk.npz``)
"""

import numpy as np

F32 = np.float32


def conv1d(x, w, b=None, padding=0):
    """x (Cin, L), w (Cout, Cin, K) -> (Cout, L + 2p - K + 1), zero padding."""
    cin, L = x.shape
    cout, _, K = w.shape
    xp = np.pad(x, ((0, 0), (padding, padding))) if padding else x
    Lo = xp.shape[1] - K + 1
    cols = np.stack([xp[:, k:k + Lo] for k in range(K)], axis=1)  # (Cin, K, Lo)
    y = w.reshape(cout, cin * K).astype(F32) @ cols.reshape(cin * K, Lo)
    if b is not None:
        y = y + b[:, None]
    return y.astype(F32)


def layer_norm(x, g, b, eps=1e-4):
    m = x.mean(0, keepdims=True)
    v = ((x - m) ** 2).mean(0, keepdims=True)
    return ((x - m) / np.sqrt(v + F32(eps)) * g.reshape(-1, 1) + b.reshape(-1, 1)).astype(F32)


def wn(sd, name):
    if name + ".weight" in sd:
        return sd[name + ".weight"]
    v, g = sd[name + ".weight_v"].astype(np.float64), sd[name + ".weight_g"].astype(np.float64)
    n = np.sqrt((v ** 2).reshape(v.shape[0], -1).sum(1)).reshape(-1, *([1] * (v.ndim - 1)))
    return (v / n * g).astype(F32)


class GlowOracle:
    def __init__(self, sd, enc_layers=9, flows=12, wn_layers=4, encoder_type="gatedconv"):
        self.sd = {k: np.asarray(v, F32) if np.asarray(v).dtype != np.int64 else np.asarray(v) for k, v in sd.items()}
        self.enc_layers, self.flows, self.wn_layers = enc_layers, flows, wn_layers
        self.encoder_type = encoder_type

    def _bn(self, x, name, eps=1e-5):
        sd = self.sd
        sc = sd[name + ".weight"] / np.sqrt(sd[name + ".running_var"] + F32(eps))
        return ((x - sd[name + ".running_mean"][:, None]) * sc[:, None] + sd[name + ".bias"][:, None]).astype(F32)

    def _tdsep(self, x):
        """encoder.py:118-121 with use_prenet: ConvLayerNorm (glow.py:43-50) then the
        TimeDepthSeparableConvBlock (time_depth_sep_conv.py:51-63,93-96); B = 1, so masks are 1."""
        sd = self.sd
        H = x.shape[0]
        x = self._prenet(x)
        for i in range(self.enc_layers):
            q = f"encoder.encoder.layers.{i}."
            h = self._bn(conv1d(x, sd[q + "time_conv.weight"], sd[q + "time_conv.bias"]), q + "norm1")
            h = (h[:H] * (F32(1) / (F32(1) + np.exp(-h[H:])))).astype(F32)               # GLU
            wd = sd[q + "depth_conv.weight"][:, 0, :]                                      # (H, 5)
            hp = np.pad(h, ((0, 0), (2, 2)))
            L = h.shape[1]
            d = sum(wd[:, k:k + 1] * hp[:, k:k + L] for k in range(5)) + sd[q + "depth_conv.bias"][:, None]
            d = self._bn(d.astype(F32), q + "norm2")
            d = (d * (F32(1) / (F32(1) + np.exp(-d)))).astype(F32)                         # x * sigmoid(x)
            o = self._bn(conv1d(d, sd[q + "time_conv2.weight"], sd[q + "time_conv2.bias"]), q + "norm3")
            x = (x + o).astype(F32)
        return x

    def _prenet(self, x):
        """ConvLayerNorm (glow.py:43-50): 3 x (conv k5 -> LayerNorm -> ReLU), x + proj(.)."""
        sd = self.sd
        h = x
        for i in range(3):
            p = "encoder.pre."
            h = conv1d(h, sd[p + f"conv_layers.{i}.weight"], sd[p + f"conv_layers.{i}.bias"], 2)
            h = np.maximum(layer_norm(h, sd[p + f"norm_layers.{i}.gamma"], sd[p + f"norm_layers.{i}.beta"]), F32(0))
        return (x + conv1d(h, sd["encoder.pre.proj.weight"], sd["encoder.pre.proj.bias"])).astype(F32)

    def _transformer(self, x, heads=2):
        """Transformer.forward (transformer.py:307-319) without relative-position tables: B = 1, so
        the attention mask is all ones."""
        sd = self.sd
        H, T = x.shape
        dk = H // heads
        L = len([k for k in sd if k.endswith(".conv_q.weight")])
        for i in range(L):
            a = f"encoder.encoder.attn_layers.{i}."
            q = conv1d(x, sd[a + "conv_q.weight"], sd[a + "conv_q.bias"])
            k = conv1d(x, sd[a + "conv_k.weight"], sd[a + "conv_k.bias"])
            v = conv1d(x, sd[a + "conv_v.weight"], sd[a + "conv_v.bias"])
            o = np.zeros_like(x)
            for hh in range(heads):
                sl = slice(hh * dk, (hh + 1) * dk)
                sc = (q[sl].T @ k[sl] / F32(np.sqrt(dk))).astype(F32)          # (T_t, T_s)
                sc = np.exp(sc - sc.max(1, keepdims=True))
                p = (sc / sc.sum(1, keepdims=True)).astype(F32)
                o[sl] = (v[sl] @ p.T).astype(F32)
            y = conv1d(o, sd[a + "conv_o.weight"], sd[a + "conv_o.bias"])
            x = layer_norm((x + y).astype(F32), sd[f"encoder.encoder.norm_layers_1.{i}.gamma"],
                           sd[f"encoder.encoder.norm_layers_1.{i}.beta"])
            f = f"encoder.encoder.ffn_layers.{i}."
            h = np.maximum(conv1d(x, sd[f + "conv_1.weight"], sd[f + "conv_1.bias"], 1), F32(0))
            y = conv1d(h, sd[f + "conv_2.weight"], sd[f + "conv_2.bias"], 1)
            x = layer_norm((x + y).astype(F32), sd[f"encoder.encoder.norm_layers_2.{i}.gamma"],
                           sd[f"encoder.encoder.norm_layers_2.{i}.beta"])
        return x

    def speaker(self, spk):
        """F.normalize(emb_g(spk)) (glow_tts.py:159-161): x / max(||x||_2, 1e-12), shape (c_in,)."""
        e = self.sd["emb_g.weight"][int(spk)]
        n = np.sqrt(np.sum(e.astype(np.float64) ** 2))
        return (e / F32(max(n, 1e-12))).astype(F32)

    def encode(self, ids, g=None):
        sd = self.sd
        H = sd["encoder.emb.weight"].shape[1]
        x = (sd["encoder.emb.weight"][ids] * F32(np.sqrt(H))).T.astype(F32)        # (H, T)
        if self.encoder_type == "time-depth-separable":
            x = self._tdsep(x)
        elif self.encoder_type == "transformer":
            x = self._transformer(self._prenet(x))
        for i in range(self.enc_layers if self.encoder_type == "gatedconv" else 0):
            p = f"encoder.encoder."
            o = conv1d(x, sd[p + f"conv_layers.{i}.weight"], sd[p + f"conv_layers.{i}.bias"], 2)
            o = layer_norm(o, sd[p + f"norm_layers.{i}.gamma"], sd[p + f"norm_layers.{i}.beta"])
            a, gate = o[:H], o[H:]
            x = (x + a * (F32(1) / (F32(1) + np.exp(-gate)))).astype(F32)
        o_mean = conv1d(x, sd["encoder.proj_m.weight"], sd["encoder.proj_m.bias"])
        d = "encoder.duration_predictor."
        x_dp = x if g is None else np.concatenate([x, np.repeat(g[:, None], x.shape[1], 1)], 0)
        h = np.maximum(conv1d(x_dp, sd[d + "conv_1.weight"], sd[d + "conv_1.bias"], 1), F32(0))
        h = layer_norm(h, sd[d + "norm_1.gamma"], sd[d + "norm_1.beta"])
        h = np.maximum(conv1d(h, sd[d + "conv_2.weight"], sd[d + "conv_2.bias"], 1), F32(0))
        h = layer_norm(h, sd[d + "norm_2.gamma"], sd[d + "norm_2.beta"])
        logw = conv1d(h, sd[d + "proj.weight"], sd[d + "proj.bias"])[0]
        return o_mean, logw

    @staticmethod
    def durations(logw, length_scale=1.0):
        w_ceil = np.ceil(((np.exp(logw) - F32(1)) * F32(length_scale)).astype(F32))
        return w_ceil, max(int(w_ceil.sum()), 1)

    def inference(self, ids, noise=None, noise_scale=0.66, length_scale=1.0, spk=None):
        """one utterance: (y (80, 2*floor(Ty/2)), y_mean (80, Ty), attn (Ty, Tx), logw (Tx,), Ty);
        ``spk``: speaker index into emb_g (multi-speaker models)"""
        sd = self.sd
        g = None if spk is None else self.speaker(spk)
        o_mean, logw = self.encode(np.asarray(ids), g)
        w_ceil, Ty = self.durations(logw, length_scale)
        cum = np.cumsum(w_ceil)
        j = np.arange(Ty, dtype=F32)[None, :]
        path = (j < cum[:, None]).astype(F32)
        path = path - np.concatenate([np.zeros((1, Ty), F32), path[:-1]], 0)          # (Tx, Ty)
        y_mean = (o_mean @ path).astype(F32)                                            # (80, Ty)
        z = y_mean if noise is None else (y_mean + noise[:, :Ty] * F32(noise_scale)).astype(F32)
        C = z.shape[0]
        K = Ty // 2
        x = z[:, :2 * K].reshape(C, K, 2).transpose(2, 0, 1).reshape(2 * C, K)         # squeeze
        for k in range(self.flows - 1, -1, -1):
            x = self._coupling_rev(x, f"decoder.flows.{3 * k + 2}.", g)
            x = self._invconv_rev(x, sd[f"decoder.flows.{3 * k + 1}.weight"])
            a = f"decoder.flows.{3 * k}."
            x = ((x - sd[a + "bias"].reshape(-1, 1)) * np.exp(-sd[a + "logs"].reshape(-1, 1))).astype(F32)
        y = x.reshape(2, C, K).transpose(1, 2, 0).reshape(C, 2 * K)                    # unsqueeze
        return y.astype(F32), y_mean, path.T.copy(), logw, Ty

    def _coupling_rev(self, x, p, g=None):
        sd = self.sd
        C = x.shape[0] // 2
        x0, x1 = x[:C], x[C:]
        h = conv1d(x0, wn(sd, p + "start"), sd[p + "start.bias"])
        H = h.shape[0]
        out = np.zeros_like(h)
        gc = None if g is None else conv1d(g[:, None], wn(sd, p + "wn.cond_layer"), sd[p + "wn.cond_layer.bias"])
        for i in range(self.wn_layers):
            a = conv1d(h, wn(sd, p + f"wn.in_layers.{i}"), sd[p + f"wn.in_layers.{i}.bias"], 2)
            if gc is not None:
                a = (a + gc[2 * H * i:2 * H * (i + 1)]).astype(F32)
            acts = (np.tanh(a[:H]) * (F32(1) / (F32(1) + np.exp(-a[H:])))).astype(F32)
            rs = conv1d(acts, wn(sd, p + f"wn.res_skip_layers.{i}"), sd[p + f"wn.res_skip_layers.{i}.bias"])
            if i < self.wn_layers - 1:
                h = (h + rs[:H]).astype(F32)
                out = (out + rs[H:]).astype(F32)
            else:
                out = (out + rs).astype(F32)
        mo = conv1d(out, sd[p + "end.weight"], sd[p + "end.bias"])
        z1 = ((x1 - mo[:C]) * np.exp(-mo[C:])).astype(F32)
        return np.concatenate([x0, z1], 0)

    @staticmethod
    def _invconv_rev(x, w):
        c, t = x.shape
        winv = np.linalg.inv(w.astype(np.float64)).astype(F32)
        xs = x.reshape(2, c // 4, 2, t).transpose(0, 2, 1, 3).reshape(4, c // 4, t)
        z = np.einsum("ab,bjt->ajt", winv, xs).astype(F32)
        return z.reshape(2, 2, c // 4, t).transpose(0, 2, 1, 3).reshape(c, t)
