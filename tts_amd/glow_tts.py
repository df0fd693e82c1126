"""Drop-in ``GlowTts`` whose ``inference`` runs on MI355X through ``libttship.so``.

Mirrors ``TTS/tts/models/glow_tts.py`` as ``setup_model`` builds it for the reference configs
(``TTS/tts/utils/generic_utils.py:105-129``: transformer (6 layers, 2 heads) or time-depth-separable
(both with the ConvLayerNorm prenet) or gated-conv encoder, hidden 192,
duration predictor 256, 12 flow blocks x 4 WN layers, kernel 5, dilation 1, num_sqz 2,
num_splits 4, mean_only): the constructor signature, the checkpoint keys (``encoder.*``,
``decoder.flows.*``), the ``noise_scale`` / ``length_scale`` attributes and
``inference(x, x_lengths, g=None)`` returning ``(y, logdet, y_mean, y_log_scale, attn, o_dur_log,
o_attn_dur)`` (``:166-193``). Batched rows are independent; row i equals the B = 1 call.

Multi-speaker models (``num_speakers > 1``, ``c_in_channels > 0``, built directly as the reference
allows; ``setup_model`` itself passes ``c_in_channels=0``) take ``g`` as a (B,) LongTensor of speaker
ids: ``emb_g`` (``:97-99``), ``g = F.normalize(emb_g(g))`` (``:159-161``), the duration predictor over
``[x; g]`` (``layers/glow_tts/encoder.py:131-135``) and each WN layer's slice of ``cond_layer(g)``
added before its gate (``layers/glow_tts/glow.py:119-130``). Misuse fails as the reference does: g
for a model without ``emb_g`` or ``cond_layer`` raises AttributeError, no g for a model built with
``c_in_channels > 0`` raises RuntimeError.

The prior sample ``z = y_mean + exp(y_log_scale) * randn * noise_scale`` draws its noise with torch
on the model's device (``torch.randn_like`` in the reference); pass ``noise=`` to fix it.
"""

from typing import Optional

import numpy as np
import torch
from torch import nn

from ._lib import get_engine
from .params import host_tensors, new_token, populate
from .spec import GlowConfig, glow_spec


class GlowTts(nn.Module):
    def __init__(self, num_chars, hidden_channels=192, filter_channels=768, filter_channels_dp=256, out_channels=80,
                 kernel_size=3, num_heads=2, num_layers_enc=6, dropout_p=0.1, num_flow_blocks_dec=12,
                 kernel_size_dec=5, dilation_rate=1, num_block_layers=4, dropout_p_dec=0., num_speakers=0,
                 c_in_channels=0, num_splits=4, num_sqz=2, sigmoid_scale=False, rel_attn_window_size=None,
                 input_length=None, mean_only=True, hidden_channels_enc=None, hidden_channels_dec=None,
                 use_encoder_prenet=False, encoder_type="gatedconv"):
        super().__init__()
        bad = []
        if encoder_type.lower() not in ("gatedconv", "time-depth-separable", "transformer"):
            bad.append(f"encoder_type={encoder_type}")
        if encoder_type.lower() in ("time-depth-separable", "transformer") and not use_encoder_prenet:
            bad.append(f"{encoder_type} encoder without the prenet")
        if encoder_type.lower() == "transformer" and (rel_attn_window_size is not None or input_length is not None
                                                      or num_heads * 96 != hidden_channels or filter_channels != 768
                                                      or kernel_size != 3):
            bad.append("transformer options other than setup_model's")
        if hidden_channels != 192 or (hidden_channels_enc or 192) != 192 or (hidden_channels_dec or 192) != 192:
            bad.append("hidden channels != 192")
        if filter_channels_dp != 256 or out_channels != 80 or kernel_size != 3 or kernel_size_dec != 5:
            bad.append("non-reference layer sizes")
        if dilation_rate != 1 or num_splits != 4 or num_sqz != 2 or sigmoid_scale or not mean_only:
            bad.append("non-reference flow options")
        if c_in_channels < 0:
            bad.append("c_in_channels < 0")
        if bad:
            raise NotImplementedError("tts_amd GlowTts implements the reference configs only: " + ", ".join(bad))
        self.num_chars = num_chars
        self.cfg = GlowConfig(num_chars=num_chars, num_layers_enc=num_layers_enc,
                              num_flow_blocks_dec=num_flow_blocks_dec, num_block_layers=num_block_layers,
                              encoder_type=encoder_type.lower(), num_speakers=num_speakers,
                              c_in_channels=c_in_channels)
        self.noise_scale = 0.66
        self.length_scale = 1.
        populate(self, glow_spec(self.cfg))
        self._version = 0
        self._token = new_token()

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

    def store_inverse(self):  # the library inverts InvConvNear and folds weight norm at load
        pass

    def forward(self, *args, **kwargs):
        raise NotImplementedError("training forward is out of scope; use inference()")

    def _sync(self, eng):
        key = (self._token, self._version)
        if eng.glow_key != key:
            c = self.cfg
            enc_layers = c.num_layers_enc if c.encoder_type == "transformer" else 3 + c.num_layers_enc
            eng.load_glow(host_tensors(self), c.num_chars, enc_layers, c.num_flow_blocks_dec,
                          c.num_block_layers)
            eng.glow_key = key

    @torch.no_grad()
    def inference(self, x, x_lengths, g=None, noise: Optional[torch.Tensor] = None):
        spk = None
        if g is not None:
            if self.cfg.num_speakers <= 1:
                raise AttributeError("'GlowTts' object has no attribute 'emb_g'")
            if not self.cfg.c_in_channels:
                raise AttributeError("'WN' object has no attribute 'cond_layer'")
            spk = np.asarray(torch.as_tensor(g).cpu(), np.int64).reshape(-1)
            if spk.min() < 0 or spk.max() >= self.cfg.num_speakers:
                raise IndexError("index out of range in self")  # nn.Embedding's message
        elif self.cfg.c_in_channels:
            raise RuntimeError(f"the duration predictor expects {192 + self.cfg.c_in_channels} input channels "
                               "(c_in_channels > 0): pass g")
        dev = self.encoder.emb.weight.device
        eng = get_engine(dev)
        with eng.lock:  # encode and decode share the context's Glow workspace
            self._sync(eng)
            x = torch.as_tensor(x).to(dev, torch.int64)
            if x.dim() == 1:
                x = x[None]
            x = x.contiguous()
            B, T = x.shape
            lens = np.asarray(torch.as_tensor(x_lengths).cpu(), np.int64).reshape(-1)
            if len(lens) != B or lens.min() < 1 or lens.max() > T:
                raise ValueError("x_lengths must have B entries in [1, T]")
            if B > 64:
                raise ValueError("at most 64 utterances per call")
            if spk is not None and len(spk) != B:
                raise ValueError("g must hold one speaker id per utterance")
            ylens = eng.glow_encode(x, lens, float(self.length_scale), spk)
            Ty = int(ylens.max())
            if noise is None:
                noise = torch.randn(B, 80, Ty, device=dev)
            noise = torch.as_tensor(noise).to(dev, torch.float32)[:, :, :Ty].contiguous()
            if noise.shape != (B, 80, Ty):
                raise ValueError(f"noise must be (B, 80, >= {Ty})")
            y = torch.empty(B, 80, 2 * (Ty // 2), device=dev)
            y_mean = torch.empty(B, 80, Ty, device=dev)
            attn = torch.empty(B, Ty, T, device=dev)
            logw = torch.empty(B, 1, T, device=dev)
            eng.glow_decode(noise, float(self.noise_scale), Ty, y, y_mean, attn, logw)
        x_mask = (torch.arange(T, device=dev)[None] < torch.as_tensor(lens, device=dev)[:, None]).float()[:, None]
        o_attn_dur = torch.log(1 + attn.sum(1, keepdim=True)) * x_mask
        self.last_y_lengths = ylens
        return y, None, y_mean, torch.zeros_like(y_mean), attn, logw * x_mask, o_attn_dur
