"""ORACLE / CPU BASELINE (test infrastructure only): PyTorch-CPU restatement of the reference
Tacotron2-DDC + MB-MelGAN inference path as the same ATen op sequence the reference runs
("the build's own PyTorch-CPU restatement of the reference math"). Only ``tests/``
and ``bench.py``'s ``cpu_baseline`` leg may import it; the product path never does.

It exists because the reference never travels to the GPU box: bench.py times THIS on the box's
host cores as the reference's CPU path. ``tools/cpu_baseline_check.py`` times it beside the
imported reference in the build container (profiles/r03/cpu_baseline_check_r*.json), and
``tests/test_oracle_golden.py`` pins its outputs to the reference fixtures.

Op sequence followed (paths relative to the reference checkout):

* ``TTS/tts/models/tacotron2.py:142-163``  embedding -> encoder -> decoder -> postnet + residual
* ``TTS/tts/layers/tacotron2.py:9-44,112-119``  conv1d k5 + BatchNorm(eval) + ReLU x3, BiLSTM (aten::lstm)
* ``TTS/tts/layers/tacotron2.py:217-233,259-298,335-374``  states, decode step (aten::lstm_cell x2,
  location-sensitive attention, projection, stopnet), AR loop with the B=1 stop rule
* ``TTS/tts/layers/common_layers.py:76-82,90-110,268-278,325-372``  prenet, location layer, sigmoid norm
* ``TTS/vocoder/models/melgan_generator.py:28-89``, ``TTS/vocoder/layers/melgan.py:5-39``  generator
* ``TTS/vocoder/layers/pqmf.py:51-56``  PQMF synthesis (conv_transpose1d zero-insert, conv1d G)
"""

import torch
import torch.nn.functional as F


def _t(v):
    return torch.as_tensor(v).float().contiguous()


class TacoTorchCPU:
    """Tacotron2-DDC inference (location-sensitive attention, sigmoid or softmax norm, no speakers)
    at B = 1, float32 ATen on the CPU."""

    def __init__(self, sd, attn_norm="sigmoid", r_init=7):
        self.w = {k: _t(v) for k, v in sd.items() if not k.startswith("coarse_decoder.") and
                  not k.endswith("num_batches_tracked")}
        self.attn_norm = attn_norm
        self.r_init = r_init
        w = self.w
        self.lstm_params = [w[f"encoder.lstm.{n}_l0{s}"] for s in ("", "_reverse")
                            for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]

    def _conv_bn(self, p, x, act):
        w = self.w
        x = F.conv1d(x, w[p + ".convolution1d.weight"], w[p + ".convolution1d.bias"], padding=2)
        x = F.batch_norm(x, w[p + ".batch_normalization.running_mean"], w[p + ".batch_normalization.running_var"],
                         w[p + ".batch_normalization.weight"], w[p + ".batch_normalization.bias"], False, 0.1, 1e-5)
        return torch.relu(x) if act == "relu" else torch.tanh(x) if act == "tanh" else x

    def encoder(self, ids):
        x = F.embedding(ids, self.w["embedding.weight"]).transpose(1, 2)          # (1, 512, T)
        for i in range(3):
            x = self._conv_bn(f"encoder.convolutions.{i}", x, "relu")
        x = x.transpose(1, 2)                                                      # (1, T, 512)
        h0 = torch.zeros(2, 1, 256)
        out, _, _ = torch.lstm(x, (h0, h0), self.lstm_params, True, 1, 0.0, False, True, True)
        return out                                                                 # (1, T, 512)

    def decoder(self, enc, r, max_steps, thr=0.5):
        w = self.w
        d = "decoder."
        a = d + "attention."
        T = enc.shape[1]
        pin = F.linear(enc, w[a + "inputs_layer.linear_layer.weight"])            # (1, T, 128)
        q = qc = h = c = torch.zeros(1, 1024)
        ctx = torch.zeros(1, enc.shape[2])
        alpha = torch.zeros(1, T)
        alpha_cum = torch.zeros(1, T)
        mem = torch.zeros(1, 80)
        outs, stops, aligns = [], [], []
        while True:
            m = mem
            for i in range(2):
                m = torch.relu(F.linear(m, w[d + f"prenet.linear_layers.{i}.linear_layer.weight"]))
            q, qc = torch.lstm_cell(torch.cat([m, ctx], -1), (q, qc), w[d + "attention_rnn.weight_ih"],
                                    w[d + "attention_rnn.weight_hh"], w[d + "attention_rnn.bias_ih"],
                                    w[d + "attention_rnn.bias_hh"])
            pq = F.linear(q, w[a + "query_layer.linear_layer.weight"]).unsqueeze(1)
            loc = F.conv1d(torch.stack([alpha, alpha_cum], 1), w[a + "location_layer.location_conv1d.weight"],
                           padding=15).transpose(1, 2)
            loc = F.linear(loc, w[a + "location_layer.location_dense.linear_layer.weight"])
            e = F.linear(torch.tanh(pq + loc + pin), w[a + "v.linear_layer.weight"],
                         w[a + "v.linear_layer.bias"]).squeeze(-1)
            if self.attn_norm == "sigmoid":
                s = torch.sigmoid(e)
                alpha = s / s.sum(1, keepdim=True)
            else:
                alpha = torch.softmax(e, -1)
            alpha_cum = alpha_cum + alpha
            ctx = torch.bmm(alpha.unsqueeze(1), enc).squeeze(1)
            h, c = torch.lstm_cell(torch.cat([q, ctx], -1), (h, c), w[d + "decoder_rnn.weight_ih"],
                                   w[d + "decoder_rnn.weight_hh"], w[d + "decoder_rnn.bias_ih"],
                                   w[d + "decoder_rnn.bias_hh"])
            y = F.linear(torch.cat([h, ctx], -1), w[d + "linear_projection.linear_layer.weight"],
                         w[d + "linear_projection.linear_layer.bias"])
            logit = F.linear(torch.cat([h, y], -1), w[d + "stopnet.1.linear_layer.weight"],
                             w[d + "stopnet.1.linear_layer.bias"])
            st = torch.sigmoid(logit)
            outs.append(y[:, :80 * r])
            stops.append(st)
            aligns.append(alpha)
            if st.item() > thr and len(outs) > 1:
                break
            if len(outs) == max_steps:
                break
            mem = y[:, 80 * (r - 1):80 * r]
        dec = torch.cat(outs, 0).reshape(1, -1, 80)                                # (1, S*r, 80)
        return dec, torch.cat(stops, 0), torch.cat(aligns, 0)

    def postnet(self, dec):
        x = dec.transpose(1, 2)
        o = x
        for i in range(5):
            o = self._conv_bn(f"postnet.convolutions.{i}", o, "tanh" if i < 4 else None)
        return (x + o).transpose(1, 2)

    @torch.no_grad()
    def inference(self, ids, r, max_steps):
        """ids: 1-D int64 -> (dec (M, 80), post (M, 80), align (S, T), stop (S,)) as numpy."""
        enc = self.encoder(torch.as_tensor(ids).long().reshape(1, -1))
        dec, stop, align = self.decoder(enc, r, max_steps)
        post = self.postnet(dec)
        return dec[0].numpy(), post[0].numpy(), align.numpy(), stop[:, 0].numpy()


class MelganTorchCPU:
    """MB-MelGAN generator + PQMF synthesis (or the full-band generator with G=None) at B = 1,
    weight norm folded, float32 ATen on the CPU. ``layers`` is tts_amd.spec.melgan_layers(cfg)."""

    def __init__(self, sd, layers, pqmf_G=None):
        self.layers = layers
        self.w, self.b = {}, {}
        for l in layers:
            if l.name + ".weight_v" in sd:
                v = torch.as_tensor(sd[l.name + ".weight_v"]).double()
                g = torch.as_tensor(sd[l.name + ".weight_g"]).double()
                n = v.reshape(v.shape[0], -1).norm(dim=1).reshape((-1,) + (1,) * (v.dim() - 1))
                self.w[l.name] = (v / n * g).float()
            else:
                self.w[l.name] = _t(sd[l.name + ".weight"])
            self.b[l.name] = _t(sd[l.name + ".bias"])
        self.G = None if pqmf_G is None else _t(pqmf_G).reshape(1, -1, _t(pqmf_G).shape[-1])

    def generator(self, c):
        ls = self.layers
        x = F.conv1d(F.pad(c, (ls[0].padding, ls[0].padding), "reflect"), self.w[ls[0].name], self.b[ls[0].name])
        i = 1
        while i < len(ls) and ls[i].kind == "convT":
            l = ls[i]
            x = F.conv_transpose1d(F.leaky_relu(x, 0.2), self.w[l.name], self.b[l.name], stride=l.stride,
                                   padding=l.padding, output_padding=l.extra.get("output_padding", 0))
            i += 1
            while i < len(ls) and ls[i].kind == "res_dconv":
                dc, pw, sc = ls[i], ls[i + 1], ls[i + 2]
                h = F.pad(F.leaky_relu(x, 0.2), (dc.padding, dc.padding), "reflect")
                h = F.conv1d(h, self.w[dc.name], self.b[dc.name], dilation=dc.dilation)
                h = F.conv1d(F.leaky_relu(h, 0.2), self.w[pw.name], self.b[pw.name])
                x = F.conv1d(x, self.w[sc.name], self.b[sc.name]) + h
                i += 3
        l = ls[i]
        x = F.conv1d(F.pad(F.leaky_relu(x, 0.2), (l.padding, l.padding), "reflect"), self.w[l.name], self.b[l.name])
        return torch.tanh(x)

    @torch.no_grad()
    def inference(self, mel, pad=0):
        """mel (80, M) numpy -> waveform (256 * (M + 2 pad),) numpy."""
        c = torch.as_tensor(mel).float().unsqueeze(0)
        if pad:
            c = F.pad(c, (pad, pad), "replicate")
        x = self.generator(c)
        if self.G is not None:  # pqmf.py:51-56
            N = x.shape[1]
            updown = torch.zeros(N, N, N)
            for k in range(N):
                updown[k, k, 0] = 1.0
            x = F.conv_transpose1d(x, updown * N, stride=N)
            x = F.conv1d(x, self.G, padding=(self.G.shape[-1] - 1) // 2)
        return x.reshape(-1).numpy()


class PwganTorchCPU:
    """ParallelWaveGAN generator inference (config C4's vocoder) at B = 1, float32 ATen on the CPU:
    the same op sequence as ``oracle/pwgan_np.py`` (which it is checked against) with conv1d /
    conv2d doing the work, fast enough to check every row of a 64-row batch.

    * ``TTS/vocoder/models/parallel_wavegan_generator.py:90-125``  replicate pad, first_conv on the
      noise, upsample, residual blocks, skip sum * sqrt(1 / layers), ReLU-conv-ReLU-conv
    * ``TTS/vocoder/layers/upsample.py:5-101``  ConvUpsample: conv_in (no bias), per factor s a
      nearest stretch then a (1, 2s + 1) Conv2d with zero padding (0, s), no bias
    * ``TTS/vocoder/layers/parallel_wavegan.py:56-87``  dilated conv + conv1x1_aux, tanh * sigmoid
      gate, conv1x1_skip / conv1x1_out, (out + residual) * sqrt(0.5) ** 2 = 0.25 as the oracle folds it
    """

    def __init__(self, sd, cfg, device="cpu"):
        """``device``: where PyTorch runs these fp32 ops. The GPU tests may put this reference on the
        GPU (PyTorch's own ROCm kernels, independent of libttship) to check all 64 rows of the C4
        batch in seconds; it is pinned to the reference fixtures on the CPU (test_oracle_golden)."""
        from oracle.pwgan_np import fold_weight_norm
        self.dev = torch.device(device)
        self.w = {k: _t(v).to(self.dev) for k, v in fold_weight_norm(sd).items()}
        self.c = cfg

    def _aux(self, mel):
        """replicate pad + ConvUpsample of one utterance: (80, M) -> (1, 80, T)."""
        w, cfg = self.w, self.c
        p = cfg.inference_padding
        c = _t(mel).to(self.dev)[None]
        if p:
            c = F.pad(c, (p, p), mode="replicate")
        c = F.conv1d(c, w["upsample_net.conv_in.weight"])
        c = c[:, None]                                                         # (1, 1, 80, L)
        for i, s in enumerate(cfg.upsample_factors):
            c = F.interpolate(c, scale_factor=(1, s), mode="nearest")
            c = F.conv2d(c, w[f"upsample_net.upsample.up_layers.{2 * i + 1}.weight"], padding=(0, s))
        return c[:, 0]                                                         # (1, 80, T)

    def inference_batch(self, mels, noises, chunk=1 << 20):
        """Many utterances at once, each exactly as its own B = 1 call: the rows sit in one time axis
        separated by zero gaps of the largest dilation, and the residual stream is re-zeroed in the
        gaps after every layer, so every dilated tap past a row's end reads the zeros of B = 1 zero
        padding. The residual blocks then run as (128 x 272) x columns GEMMs over column chunks.
        mels: [(80, M_i)], noises: [(T_i,)] -> [waveform (T_i,)] numpy float32."""
        w, cfg = self.w, self.c
        G = max(cfg.dilation(i) for i in range(cfg.num_res_blocks)) * ((cfg.kernel_size - 1) // 2)
        with torch.no_grad():
            aux = [self._aux(m)[0] for m in mels]
            starts, pos = [], G
            for a in aux:
                starts.append(pos)
                pos += a.shape[1] + G
            N = pos
            c = torch.zeros(cfg.aux_channels, N, device=self.dev)
            x = torch.zeros(cfg.res_channels, N, device=self.dev)
            mask = torch.zeros(1, N, device=self.dev)
            fw, fb = w["first_conv.weight"].reshape(-1, 1), w["first_conv.bias"].reshape(-1, 1)
            for a, nz, s0 in zip(aux, noises, starts):
                n = a.shape[1]
                assert len(nz) == n, "noise length != upsampled length"
                c[:, s0:s0 + n] = a
                x[:, s0:s0 + n] = fw * _t(nz).to(self.dev)[None] + fb
                mask[:, s0:s0 + n] = 1.0
            skips = torch.zeros(cfg.skip_channels, N, device=self.dev)
            H = cfg.gate_channels // 2
            for i in range(cfg.num_res_blocks):
                q = f"conv_layers.{i}."
                d = cfg.dilation(i)
                W = w[q + "conv.weight"]                                      # (128, 64, 3): taps t-d, t, t+d
                Wc = torch.cat([W[:, :, k] for k in range(cfg.kernel_size)], 1)
                Wa, b = w[q + "conv1x1_aux.weight"][:, :, 0], w[q + "conv.bias"].reshape(-1, 1)
                Ws, bs = w[q + "conv1x1_skip.weight"][:, :, 0], w[q + "conv1x1_skip.bias"].reshape(-1, 1)
                Wo, bo = w[q + "conv1x1_out.weight"][:, :, 0], w[q + "conv1x1_out.bias"].reshape(-1, 1)
                xn = torch.zeros_like(x)
                for s0 in range(G, N - G, chunk):
                    e = min(s0 + chunk, N - G)
                    X3 = torch.cat([x[:, s0 - d:e - d], x[:, s0:e], x[:, s0 + d:e + d]], 0)
                    a = torch.addmm(b, Wc, X3) + Wa @ c[:, s0:e]
                    z = torch.tanh(a[:H]) * torch.sigmoid(a[H:])
                    skips[:, s0:e] += torch.addmm(bs, Ws, z)
                    xn[:, s0:e] = (torch.addmm(bo, Wo, z) + x[:, s0:e]) * 0.25
                x = xn * mask
            outs = []
            w1, b1 = w["last_conv_layers.1.weight"][:, :, 0], w["last_conv_layers.1.bias"].reshape(-1, 1)
            w3, b3 = w["last_conv_layers.3.weight"][:, :, 0], w["last_conv_layers.3.bias"].reshape(-1, 1)
            for a, s0 in zip(aux, starts):
                n = a.shape[1]
                h = torch.relu(skips[:, s0:s0 + n] * (1.0 / cfg.num_res_blocks) ** 0.5)
                h = torch.relu(torch.addmm(b1, w1, h))
                outs.append(torch.addmm(b3, w3, h)[0].cpu().numpy())
        return outs

    def inference(self, mel, noise):
        """mel (80, M), noise (T,) with T = (M + 2 pad) * 256 -> waveform (T,) numpy float32."""
        w, cfg = self.w, self.c
        with torch.no_grad():
            c = self._aux(mel)                                                 # (1, 80, T)
            x = F.conv1d(_t(noise).to(self.dev)[None, None], w["first_conv.weight"], w["first_conv.bias"])
            skips = 0
            H = cfg.gate_channels // 2
            for i in range(cfg.num_res_blocks):
                q = f"conv_layers.{i}."
                d = cfg.dilation(i)
                a = F.conv1d(x, w[q + "conv.weight"], w[q + "conv.bias"], padding=(cfg.kernel_size - 1) // 2 * d,
                             dilation=d)
                a = a + F.conv1d(c, w[q + "conv1x1_aux.weight"])
                z = torch.tanh(a[:, :H]) * torch.sigmoid(a[:, H:])
                s = F.conv1d(z, w[q + "conv1x1_skip.weight"], w[q + "conv1x1_skip.bias"])
                x = (F.conv1d(z, w[q + "conv1x1_out.weight"], w[q + "conv1x1_out.bias"]) + x) * 0.25
                skips = skips + s
            h = torch.relu(skips * (1.0 / cfg.num_res_blocks) ** 0.5)
            h = torch.relu(F.conv1d(h, w["last_conv_layers.1.weight"], w["last_conv_layers.1.bias"]))
            y = F.conv1d(h, w["last_conv_layers.3.weight"], w["last_conv_layers.3.bias"])
        return y[0, 0].cpu().numpy()
