"""Drop-in MelGAN-family generators whose ``inference`` runs on MI355X via ``libttship.so``.

Mirrors ``TTS/vocoder/models/melgan_generator.py:8-97`` (constructor, ``layers.N`` checkpoint
keys with ``weight_g`` / ``weight_v`` before ``remove_weight_norm()``, ``inference_padding``),
``multiband_melgan_generator.py:7-39`` (``pqmf_layer`` buffers, PQMF synthesis) and
``fullband_melgan_generator.py``. Batching (new, optional): ``inference(c, lengths=...)`` on
(B, 80, M) padded mels; row b equals the reference call on ``c[b:b+1, :, :lengths[b]]``,
zero past ``hop * (lengths[b] + 2 * inference_padding)`` samples.
"""

from typing import Optional, Sequence

import numpy as np
import torch
from torch import nn

from ._lib import get_engine
from .params import Container, host_tensors, new_token, populate
from .pqmf import pqmf_filters
from .spec import MelganConfig, PwganConfig, melgan_layers, melgan_spec, pwgan_spec


class PQMF(Container):
    """Buffers of ``TTS/vocoder/layers/pqmf.py:10-43``; synthesis runs in the HIP library."""

    def __init__(self, N=4, taps=62, cutoff=0.15, beta=9.0):
        super().__init__()
        self.N, self.taps, self.cutoff, self.beta = N, taps, cutoff, beta
        H, G, updown = pqmf_filters(N, taps, cutoff, beta)
        self.register_buffer("H", torch.from_numpy(H))
        self.register_buffer("G", torch.from_numpy(G))
        self.register_buffer("updown_filter", torch.from_numpy(updown))

    @torch.no_grad()
    def synthesis(self, x):
        eng = get_engine(x.device)
        x = x.to(torch.float32).contiguous()
        B, N, L = x.shape
        if N != self.N:
            raise ValueError(f"expected {self.N} subbands, got {N}")
        y = torch.empty(B, 1, N * L, device=x.device, dtype=torch.float32)
        G = self.G.to(x.device, torch.float32).reshape(N, -1).contiguous()
        with eng.lock:
            eng.pqmf_synthesis(x, G, y)
        return y

    def analysis(self, x):  # training-only path in the reference (pqmf.py:48-49)
        raise NotImplementedError("PQMF analysis is training-only and out of scope")


class MelganGenerator(nn.Module):
    _use_pqmf = False

    def __init__(self, in_channels=80, out_channels=1, proj_kernel=7, base_channels=512,
                 upsample_factors=(8, 8, 2, 2), res_kernel=3, num_res_blocks=3):
        super().__init__()
        if proj_kernel != 7 or res_kernel != 3:
            raise NotImplementedError("only proj_kernel=7, res_kernel=3 (the reference configs) are built")
        if any(u % 2 or u > 8 for u in upsample_factors):
            raise NotImplementedError("upsample factors must be even and <= 8")
        if in_channels % 16 or base_channels % (16 << len(upsample_factors)):
            raise NotImplementedError("channel counts must keep multiples of 16 at every stage")
        self.cfg = MelganConfig(in_channels=in_channels, out_channels=out_channels, proj_kernel=proj_kernel,
                                base_channels=base_channels, upsample_factors=tuple(upsample_factors),
                                res_kernel=res_kernel, num_res_blocks=num_res_blocks, pqmf=False)
        self.inference_padding = 2
        self._wn = True
        populate(self, melgan_spec(self.cfg, weight_norm=True))
        self._version = 0
        self._token = new_token()

    @property
    def hop(self):
        return int(np.prod(self.cfg.upsample_factors)) * (self.cfg.out_channels if self._use_pqmf else 1)

    def load_state_dict(self, state_dict, strict=True, **kw):
        res = super().load_state_dict(state_dict, strict=strict, **kw)
        self._version += 1
        return res

    def _apply(self, fn, *args, **kwargs):
        res = super()._apply(fn, *args, **kwargs)
        self._version += 1
        return res

    def invalidate(self):
        self._version += 1

    def remove_weight_norm(self):
        """Fold w = g * v / ||v|| (melgan_generator.py:91-97, melgan.py:41-45)."""
        if not self._wn:
            return
        for l in melgan_layers(self.cfg):
            *path, = l.name.split(".")
            m = self
            for p in path:
                m = m._modules[p]
            g, v = m.weight_g.data, m.weight_v.data
            w = torch._weight_norm(v, g, 0)
            del m._parameters["weight_g"]
            del m._parameters["weight_v"]
            m.weight = nn.Parameter(w.contiguous(), requires_grad=False)
        self._wn = False
        self._version += 1

    def forward(self, c):
        return self.inference(c)

    def _sync(self, eng):
        key = (self._token, self._version)
        if eng.melgan_key != key:
            eng.load_melgan(host_tensors(self, skip_prefixes=("pqmf_layer.H", "pqmf_layer.updown")),
                            self.cfg.in_channels, self.cfg.out_channels, self.cfg.base_channels,
                            self.cfg.upsample_factors, self.cfg.num_res_blocks, self._use_pqmf)
            eng.melgan_key = key

    def _prep(self, c, lengths, frame_major_ok=False):
        dev = self.layers._modules["1"].bias.device
        eng = get_engine(dev)
        c = torch.as_tensor(c).to(dev, torch.float32)
        if c.dim() == 2:
            c = c[None]
        # frame_major_ok: a (B, M, C) tensor viewed as (B, C, M) (e.g. postnet_out.transpose(1, 2)) is
        # read in place by tts_melgan_infer_strided instead of being copied
        B, C, M = c.shape
        frame_major = (frame_major_ok and c.stride(1) == 1 and c.stride(2) == C and c.stride(0) == M * C
                       and C % 4 == 0 and c.data_ptr() % 16 == 0)
        if not frame_major:
            c = c.contiguous()
        if C != self.cfg.in_channels:
            raise ValueError(f"expected {self.cfg.in_channels} mel channels, got {C}")
        lens = np.full(B, M, np.int64) if lengths is None else np.asarray(torch.as_tensor(lengths).cpu(), np.int64)
        pad = int(self.inference_padding)
        if (lens + 2 * pad < 4).any():
            raise RuntimeError("ReflectionPad1d: padding (3) must be < input length; need frames + 2*padding >= 4")
        # ResidualStack(dilation 3^k) pads by its dilation (vocoder/layers/melgan.py:14-20): the first
        # stage's length must exceed the largest one, as torch's ReflectionPad1d requires
        dmax = 3 ** (self.cfg.num_res_blocks - 1)
        if ((lens + 2 * pad) * int(self.cfg.upsample_factors[0]) <= dmax).any():
            raise RuntimeError(f"ReflectionPad1d: padding ({dmax}) must be < input length of the first residual stack")
        return eng, c, lens, pad

    @torch.no_grad()
    def generator(self, c, lengths: Optional[Sequence[int]] = None):
        """``self.layers(pad(c))``: (B, out_channels, up * (M + 2p))."""
        eng, c, lens, pad = self._prep(c, lengths)
        B, _, M = c.shape
        up = int(np.prod(self.cfg.upsample_factors))
        out = torch.empty(B, self.cfg.out_channels, up * (M + 2 * pad), device=c.device)
        with eng.lock:
            self._sync(eng)
            eng.melgan_generator(c, lens, pad, out)
        return out

    @torch.no_grad()
    def inference(self, c, lengths: Optional[Sequence[int]] = None):
        return self.generator(c, lengths)


class MultibandMelganGenerator(MelganGenerator):
    _use_pqmf = True

    def __init__(self, in_channels=80, out_channels=4, proj_kernel=7, base_channels=384,
                 upsample_factors=(2, 8, 2, 2), res_kernel=3, num_res_blocks=3):
        super().__init__(in_channels=in_channels, out_channels=out_channels, proj_kernel=proj_kernel,
                         base_channels=base_channels, upsample_factors=upsample_factors, res_kernel=res_kernel,
                         num_res_blocks=num_res_blocks)
        self.pqmf_layer = PQMF(N=4, taps=62, cutoff=0.15, beta=9.0)
        self.cfg.pqmf = True
        self._version += 1

    def pqmf_synthesis(self, x):
        return self.pqmf_layer.synthesis(x)

    def pqmf_analysis(self, x):
        return self.pqmf_layer.analysis(x)

    @torch.no_grad()
    def inference(self, cond_features, lengths: Optional[Sequence[int]] = None):
        eng, c, lens, pad = self._prep(cond_features, lengths, frame_major_ok=True)
        B, _, M = c.shape
        wav = torch.empty(B, 1, self.hop * (M + 2 * pad), device=c.device)
        with eng.lock:
            self._sync(eng)
            eng.melgan_infer(c, lens, pad, wav)
        return wav


class FullbandMelganGenerator(MelganGenerator):
    def __init__(self, in_channels=80, out_channels=1, proj_kernel=7, base_channels=512,
                 upsample_factors=(2, 8, 2, 2), res_kernel=3, num_res_blocks=4):
        super().__init__(in_channels=in_channels, out_channels=out_channels, proj_kernel=proj_kernel,
                         base_channels=base_channels, upsample_factors=upsample_factors, res_kernel=res_kernel,
                         num_res_blocks=num_res_blocks)


class ParallelWaveganGenerator(nn.Module):
    """``TTS/vocoder/models/parallel_wavegan_generator.py:9-158`` for the configuration
    ``setup_generator`` builds (64 res / 128 gate / 64 skip / 80 aux channels, kernel 3, bias,
    no dropout at inference): constructor, checkpoint keys (weight_g / weight_v until
    ``remove_weight_norm()``), ``inference(c)`` -> (B, 1, hop * (M + 2 * inference_padding)).

    The prior noise is ``torch.randn([B, 1, T])`` on the CPU generator, as the reference draws it
    (``:96``), so a seeded call reproduces the reference's noise; pass ``noise=`` to fix it.
    Batching (new, optional): ``lengths=`` gives per-row mel frames of a padded batch."""

    def __init__(self, in_channels=1, out_channels=1, kernel_size=3, num_res_blocks=30, stacks=3, res_channels=64,
                 gate_channels=128, skip_channels=64, aux_channels=80, dropout=0.0, bias=True, use_weight_norm=True,
                 upsample_factors=(4, 4, 4, 4), inference_padding=2):
        super().__init__()
        if (in_channels, out_channels, kernel_size, res_channels, gate_channels, skip_channels, aux_channels) != \
                (1, 1, 3, 64, 128, 64, 80) or not bias:
            raise NotImplementedError("tts_amd ParallelWaveganGenerator implements the reference configuration "
                                      "(1/1 channels, kernel 3, res 64, gate 128, skip 64, aux 80, bias)")
        if num_res_blocks % stacks:
            raise ValueError("num_res_blocks must be a multiple of stacks")
        self.cfg = PwganConfig(num_res_blocks=num_res_blocks, stacks=stacks, upsample_factors=tuple(upsample_factors),
                               inference_padding=inference_padding)
        self.in_channels, self.out_channels, self.aux_channels = in_channels, out_channels, aux_channels
        self.num_res_blocks, self.stacks, self.kernel_size = num_res_blocks, stacks, kernel_size
        self.upsample_factors = list(upsample_factors)
        self.upsample_scale = int(np.prod(upsample_factors))
        self.inference_padding = inference_padding
        self.dropout = dropout
        self._wn = use_weight_norm
        populate(self, pwgan_spec(self.cfg, weight_norm=use_weight_norm))
        self._version = 0
        self._token = new_token()

    @property
    def hop(self):
        return self.upsample_scale

    def load_state_dict(self, state_dict, strict=True, **kw):
        res = super().load_state_dict(state_dict, strict=strict, **kw)
        self._version += 1
        return res

    def _apply(self, fn, *args, **kwargs):
        res = super()._apply(fn, *args, **kwargs)
        self._version += 1
        return res

    def invalidate(self):
        self._version += 1

    def remove_weight_norm(self):
        """Fold w = g * v / ||v|| for every weight-normed conv (parallel_wavegan_generator.py:127-135)."""
        if not self._wn:
            return
        for name, shape, kind in pwgan_spec(self.cfg, weight_norm=True):
            if not name.endswith(".weight_v"):
                continue
            path = name[:-len(".weight_v")].split(".")
            m = self
            for p in path:
                m = m._modules[p]
            w = torch._weight_norm(m.weight_v.data, m.weight_g.data, 0)
            del m._parameters["weight_g"]
            del m._parameters["weight_v"]
            m.weight = nn.Parameter(w.contiguous(), requires_grad=False)
        self._wn = False
        self._version += 1

    def _sync(self, eng):
        key = (self._token, self._version)
        if eng.pwgan_key != key:
            eng.load_pwgan(host_tensors(self), self.cfg.num_res_blocks, self.cfg.stacks, self.cfg.upsample_factors)
            eng.pwgan_key = key

    def forward(self, c):
        raise NotImplementedError("training forward is out of scope; use inference()")

    @torch.no_grad()
    def inference(self, c, lengths: Optional[Sequence[int]] = None, noise: Optional[torch.Tensor] = None):
        dev = self.first_conv.bias.device
        eng = get_engine(dev)
        c = torch.as_tensor(c).to(dev, torch.float32)
        if c.dim() == 2:
            c = c[None]
        c = c.contiguous()
        B, C, M = c.shape
        if C != self.aux_channels:
            raise ValueError(f"expected {self.aux_channels} mel channels, got {C}")
        lens = np.full(B, M, np.int64) if lengths is None else np.asarray(torch.as_tensor(lengths).cpu(), np.int64)
        pad = int(self.inference_padding)
        T = self.hop * (M + 2 * pad)
        if noise is None:
            noise = torch.randn([B, 1, T])
        noise = torch.as_tensor(noise).to(dev, torch.float32).contiguous()
        if tuple(noise.shape) != (B, 1, T):
            raise ValueError(f"noise must be (B, 1, {T})")
        out = torch.empty(B, 1, T, device=dev)
        with eng.lock:
            self._sync(eng)
            eng.pwgan_infer(c, lens, pad, noise, out)
        return out
