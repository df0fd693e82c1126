"""ORACLE (test infrastructure only): float32 numpy restatement of the reference
Tacotron2 inference path. Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module; the product path never does.

Parity pin: checked against ``tests/golden/taco_*.npz``, which were produced by running
the reference (``TTS.tts.models.tacotron2.Tacotron2.inference``) in the build container
(``tests/golden/make_golden.py``).

Every function follows one reference op sequence, cited file:line
(paths relative to the reference checkout):

* ``TTS/tts/models/tacotron2.py:142-163``  Tacotron2.inference
* ``TTS/tts/layers/tacotron2.py:9-44``      ConvBNBlock (conv -> BN(eval) -> act)
* ``TTS/tts/layers/tacotron2.py:47-72``     Postnet
* ``TTS/tts/layers/tacotron2.py:112-119``   Encoder.inference (3 convs + BiLSTM, no packing)
* ``TTS/tts/layers/tacotron2.py:259-298``   Decoder.decode
* ``TTS/tts/layers/tacotron2.py:335-374``   Decoder.inference (AR loop, stop rule)
* ``TTS/tts/layers/common_layers.py:76-82``   Prenet.forward
* ``TTS/tts/layers/common_layers.py:90-110``  LocationLayer
* ``TTS/tts/layers/common_layers.py:268-278,325-372`` OriginalAttention (location, norm)
"""

import numpy as np

F32 = np.float32


def sigmoid(x):
    x = np.asarray(x, F32)
    with np.errstate(over="ignore"):
        return (F32(1.0) / (F32(1.0) + np.exp(-x))).astype(F32)


def conv1d(x, w, b=None, padding=0, dilation=1):
    """x (Cin, L), w (Cout, Cin, K) -> (Cout, Lout); zero padding (torch.nn.Conv1d)."""
    cin, L = x.shape
    cout, _, K = w.shape
    xp = np.pad(x, ((0, 0), (padding, padding))) if padding else x
    Lout = xp.shape[1] - dilation * (K - 1)
    cols = np.empty((cin, K, Lout), F32)
    for k in range(K):
        cols[:, k, :] = xp[:, k * dilation:k * dilation + Lout]
    y = w.reshape(cout, cin * K).astype(F32) @ cols.reshape(cin * K, Lout)
    if b is not None:
        y = y + b[:, None]
    return y.astype(F32)


def batchnorm_eval(x, p, eps=1e-5):
    """BatchNorm1d eval (tacotron2.py:30): (x - mean) / sqrt(var + eps) * w + b."""
    inv = (F32(1.0) / np.sqrt(p["running_var"].astype(F32) + F32(eps))).astype(F32)
    return ((x - p["running_mean"][:, None]) * inv[:, None] * p["weight"][:, None]
            + p["bias"][:, None]).astype(F32)


def lstm_cell(x, h, c, w_ih, w_hh, b_ih, b_hh):
    """torch.nn.LSTMCell: gates i, f, g, o (chunk order)."""
    gates = (x @ w_ih.T + b_ih) + (h @ w_hh.T + b_hh)
    H = h.shape[-1]
    i = sigmoid(gates[..., 0:H])
    f = sigmoid(gates[..., H:2 * H])
    g = np.tanh(gates[..., 2 * H:3 * H]).astype(F32)
    o = sigmoid(gates[..., 3 * H:4 * H])
    c2 = (f * c + i * g).astype(F32)
    h2 = (o * np.tanh(c2)).astype(F32)
    return h2, c2


class TacoOracle:
    def __init__(self, sd, attn_norm="sigmoid", r_init=7, frame_channels=80, windowing=False,
                 forward_attn=False, trans_agent=False, forward_attn_mask=False, attn_type="original", attn_K=5):
        self.sd = {k: (np.asarray(v, F32) if np.asarray(v).dtype != np.int64 else np.asarray(v))
                   for k, v in sd.items()}
        self.attn_norm = attn_norm
        self.r_init = r_init
        self.F = frame_channels
        self.windowing = windowing
        self.forward_attn = forward_attn
        self.trans_agent = trans_agent
        self.forward_attn_mask = forward_attn_mask
        self.attn_type = attn_type
        self.attn_K = attn_K

    def _bn(self, prefix):
        return {k: self.sd[f"{prefix}.batch_normalization.{k}"]
                for k in ("weight", "bias", "running_mean", "running_var")}

    def conv_bn_block(self, prefix, x, act):
        """ConvBNBlock.forward (tacotron2.py:39-44); k5 'same' padding."""
        w = self.sd[f"{prefix}.convolution1d.weight"]
        b = self.sd[f"{prefix}.convolution1d.bias"]
        o = conv1d(x, w, b, padding=(w.shape[2] - 1) // 2)
        o = batchnorm_eval(o, self._bn(prefix))
        if act == "relu":
            o = np.maximum(o, F32(0))
        elif act == "tanh":
            o = np.tanh(o).astype(F32)
        return o

    # ---- encoder -------------------------------------------------------------------
    def encoder(self, ids):
        """embedding (tacotron2.py(models):144) + Encoder.inference (layers:112-119)."""
        x = self.sd["embedding.weight"][ids].T.astype(F32)          # (512, T)
        for i in range(3):
            x = self.conv_bn_block(f"encoder.convolutions.{i}", x, "relu")
        x = x.T                                                     # (T, 512)
        T = x.shape[0]
        outs = []
        for sfx, order in (("", range(T)), ("_reverse", range(T - 1, -1, -1))):
            w_ih = self.sd[f"encoder.lstm.weight_ih_l0{sfx}"]
            w_hh = self.sd[f"encoder.lstm.weight_hh_l0{sfx}"]
            b_ih = self.sd[f"encoder.lstm.bias_ih_l0{sfx}"]
            b_hh = self.sd[f"encoder.lstm.bias_hh_l0{sfx}"]
            H = w_hh.shape[1]
            h = np.zeros(H, F32)
            c = np.zeros(H, F32)
            o = np.zeros((T, H), F32)
            xin = (x @ w_ih.T + b_ih).astype(F32)                   # input projection
            for t in order:
                gates = xin[t] + (h @ w_hh.T + b_hh)
                i_ = sigmoid(gates[0:H]); f_ = sigmoid(gates[H:2 * H])
                g_ = np.tanh(gates[2 * H:3 * H]).astype(F32); o_ = sigmoid(gates[3 * H:])
                c = (f_ * c + i_ * g_).astype(F32)
                h = (o_ * np.tanh(c)).astype(F32)
                o[t] = h
            outs.append(o)
        return np.concatenate(outs, axis=1)                         # (T, 512)

    # ---- decoder -------------------------------------------------------------------
    def prenet(self, m):
        """Prenet.forward (common_layers.py:76-82), eval mode (no dropout); 'bn' type: LinearBN
        (common_layers.py:25-46) = Linear(bias=False) then BatchNorm1d in eval."""
        for i in range(2):
            p = f"decoder.prenet.linear_layers.{i}."
            m = (m @ self.sd[p + "linear_layer.weight"].T).astype(F32)
            if p + "batch_normalization.weight" in self.sd:
                m = batchnorm_eval(m[:, None], {k: self.sd[p + "batch_normalization." + k]
                                                for k in ("weight", "bias", "running_mean", "running_var")})[:, 0]
            m = np.maximum(m, F32(0)).astype(F32)
        return m

    def graves(self, query, inputs, st):
        """GravesAttention.forward (common_layers.py:150-193), eval mode (no dropout), mask None."""
        p = "decoder.attention.N_a."
        K = self.attn_K
        hid = np.maximum(query @ self.sd[p + "0.weight"].T + self.sd[p + "0.bias"], F32(0)).astype(F32)
        gbk = (hid @ self.sd[p + "2.weight"].T + self.sd[p + "2.bias"]).astype(F32)
        g, b, k = gbk[:K], gbk[K:2 * K], gbk[2 * K:]

        def softplus(x):  # torch: x above the threshold 20, log1p(exp(x)) otherwise
            return np.where(x > 20, x, np.log1p(np.exp(np.minimum(x, 20)))).astype(F32)
        sig = (softplus(b) + F32(1e-5)).astype(F32)
        mu = (st["mu"] + softplus(k)).astype(F32)
        e = np.exp(g - g.max())
        g = (e / e.sum() + F32(1e-5)).astype(F32)
        T = inputs.shape[0]
        j = np.arange(T + 1, dtype=F32) + F32(0.5)
        phi = g[:, None] * (F32(1) / (F32(1) + sigmoid((mu[:, None] - j[None, :]) / sig[:, None])))
        a = phi.astype(F32).sum(0)
        a = (a[1:] - a[:-1]).astype(F32)
        a[a == 0] = F32(1e-8)
        st["mu"] = mu
        st["alpha"] = a
        return (a @ inputs).astype(F32)

    def attention(self, query, inputs, pin, st):
        """OriginalAttention.forward (common_layers.py:325-372), location-sensitive."""
        if self.attn_type == "graves":
            return self.graves(query, inputs, st)
        p = "decoder.attention."
        cat = np.stack([st["alpha"], st["alpha_cum"]])              # (2, T)
        pq = query @ self.sd[p + "query_layer.linear_layer.weight"].T       # (128,)
        wl = self.sd[p + "location_layer.location_conv1d.weight"]
        f = conv1d(cat, wl, None, padding=(wl.shape[2] - 1) // 2)   # (32, T)
        loc = f.T @ self.sd[p + "location_layer.location_dense.linear_layer.weight"].T  # (T,128)
        e = np.tanh(pq[None, :] + loc + pin).astype(F32) @ self.sd[p + "v.linear_layer.weight"].T
        e = (e[:, 0] + self.sd[p + "v.linear_layer.bias"][0]).astype(F32)
        if self.windowing:  # apply_windowing (common_layers.py:286-300), B = 1
            w = st["win_idx"]
            back, front = w - 2, w + 6
            if back > 0:
                e[:back] = -np.inf
            if front < len(e):
                e[front:] = -np.inf
            if w == -1:
                e[0] = e.max()
            st["win_idx"] = int(np.argmax(e))
        if self.attn_norm == "softmax":
            z = np.exp(e - e.max()).astype(F32)
            a = (z / z.sum()).astype(F32)
        elif self.attn_norm == "sigmoid":
            s = sigmoid(e)
            a = (s / s.sum()).astype(F32)
        else:
            raise ValueError("Unknown value for attention norm type")
        st["alpha_cum"] = (st["alpha_cum"] + a).astype(F32)
        if self.forward_attn:  # apply_forward_attention (common_layers.py:302-323)
            prev = st["fwd_alpha"]
            shifted = np.concatenate([np.zeros(1, F32), prev[:-1]])
            a = (((F32(1) - st["u"]) * prev + st["u"] * shifted + F32(1e-8)) * a).astype(F32)
            if self.forward_attn_mask:  # :309-318, Python slice / negative-index semantics kept
                n = int(np.argmax(shifted))
                val = a.max()
                a[n + 3:] = 0
                a[:n - 1] = 0
                a[n - 2] = F32(0.01) * val
            a = (a / a.sum()).astype(F32)
            st["fwd_alpha"] = a
        st["alpha"] = a
        ctx = (a @ inputs).astype(F32)
        if self.forward_attn and self.trans_agent:  # u = sigmoid(ta([context, query]))
            ta = np.concatenate([ctx, query]) @ self.sd[p + "ta.weight"].T + self.sd[p + "ta.bias"]
            st["u"] = sigmoid(ta.astype(F32))[0]
        return ctx

    def decode(self, mem, inputs, pin, st):
        """Decoder.decode (tacotron2.py:259-298)."""
        sd = self.sd
        q_in = np.concatenate([mem, st["ctx"]])
        st["q"], st["qc"] = lstm_cell(q_in, st["q"], st["qc"], sd["decoder.attention_rnn.weight_ih"],
                                      sd["decoder.attention_rnn.weight_hh"],
                                      sd["decoder.attention_rnn.bias_ih"],
                                      sd["decoder.attention_rnn.bias_hh"])
        st["ctx"] = self.attention(st["q"], inputs, pin, st)
        d_in = np.concatenate([st["q"], st["ctx"]])
        st["h"], st["c"] = lstm_cell(d_in, st["h"], st["c"], sd["decoder.decoder_rnn.weight_ih"],
                                     sd["decoder.decoder_rnn.weight_hh"],
                                     sd["decoder.decoder_rnn.bias_ih"],
                                     sd["decoder.decoder_rnn.bias_hh"])
        hc = np.concatenate([st["h"], st["ctx"]])
        y = (hc @ sd["decoder.linear_projection.linear_layer.weight"].T
             + sd["decoder.linear_projection.linear_layer.bias"]).astype(F32)
        s_in = np.concatenate([st["h"], y])
        logit = (s_in @ sd["decoder.stopnet.1.linear_layer.weight"].T
                 + sd["decoder.stopnet.1.linear_layer.bias"]).astype(F32)[0]
        return y, st["alpha"], logit

    def decoder_inference(self, inputs, r, max_steps, stop_threshold=0.5, return_logits=False, return_state=False):
        """Decoder.inference (tacotron2.py:335-374) at B=1 (stop iff sigma>thr and t>0)."""
        F = self.F
        T = inputs.shape[0]
        pin = None if self.attn_type == "graves" else \
            (inputs @ self.sd["decoder.attention.inputs_layer.linear_layer.weight"].T).astype(F32)
        st = dict(q=np.zeros(1024, F32), qc=np.zeros(1024, F32), h=np.zeros(1024, F32), mu=np.zeros(self.attn_K, F32),
                  c=np.zeros(1024, F32), ctx=np.zeros(inputs.shape[1], F32),
                  alpha=np.zeros(T, F32), alpha_cum=np.zeros(T, F32), win_idx=-1, u=F32(0.5),
                  fwd_alpha=np.concatenate([np.ones(1, F32), np.full(T - 1, 1e-7, F32)]))
        mem = np.zeros(F, F32)                 # go frame, after _update_memory
        outs, stops, aligns, logits, t = [], [], [], [], 0
        while True:
            m = self.prenet(mem)
            y, a, lg = self.decode(m, inputs, pin, st)
            s = sigmoid(lg)
            outs.append(y[:F * r].copy()); stops.append(s); aligns.append(a.copy()); logits.append(lg)
            if s > stop_threshold and t > 0:
                break
            if len(outs) == max_steps:
                break
            mem = y[F * (r - 1):F * r]
            t += 1
        dec = np.stack(outs).reshape(-1, F)                         # (S*r, 80)
        res = (dec, np.array(stops, F32), np.stack(aligns))
        if return_logits:
            res = res + (np.array(logits, F32),)
        if return_state:  # what the reference leaves on `self` (layers/tacotron2.py:217-233)
            res = res + ({"query": st["q"], "attention_rnn_cell_state": st["qc"], "decoder_hidden": st["h"],
                          "decoder_cell": st["c"], "context": st["ctx"], "attention_weights": st["alpha"],
                          "attention_weights_cum": st["alpha_cum"]},)
        return res

    def postnet(self, dec):
        """Postnet (tacotron2.py:47-72) + residual (models/tacotron2.py:159-160); dec (M,80)."""
        x = dec.T.astype(F32)
        o = x
        for i in range(5):
            o = self.conv_bn_block(f"postnet.convolutions.{i}", o, "tanh" if i < 4 else None)
        return (x + o).T.astype(F32)

    def decoder_state(self, ids, r, max_steps, stop_threshold=0.5):
        """The decoder state after Tacotron2.inference (one utterance), as the reference keeps it."""
        enc = self.encoder(np.asarray(ids))
        return self.decoder_inference(enc, r, max_steps, stop_threshold, return_state=True)[-1]

    def inference(self, ids, r, max_steps=1000, stop_threshold=0.5, speaker=None):
        """Tacotron2.inference (models/tacotron2.py:142-163) for one utterance. ``speaker``: the
        speaker vector (learned-embedding row or external embedding) concatenated to every
        encoder output (models/tacotron2.py:152-155, tacotron_abstract.py:213-217)."""
        enc = self.encoder(np.asarray(ids))
        if speaker is not None:
            spk = np.asarray(speaker, F32).reshape(1, -1)
            enc = np.concatenate([enc, np.repeat(spk, enc.shape[0], axis=0)], axis=1).astype(F32)
        dec, stop, align = self.decoder_inference(enc, r, max_steps, stop_threshold)
        post = self.postnet(dec)
        return dec, post, align, stop
