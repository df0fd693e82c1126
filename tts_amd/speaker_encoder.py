"""Drop-in GE2E ``SpeakerEncoder`` whose ``inference`` runs on MI355X through ``libttship.so``.

Mirrors ``TTS/speaker_encoder/model.py``: the constructor signature (``:31-47``), the checkpoint
keys (``layers.{i}.lstm.*`` / ``layers.{i}.linear.weight`` with projection, ``layers.lstm.*`` /
``layers.linear.*`` without), ``inference(x)`` (``:62-68``: B x T x D mel frames -> B x proj_dim
L2-normalised embedding of the last frame) and ``compute_embedding(x, num_frames, overlap)``
(``:70-88``: the mean of the window embeddings). The windows of one utterance run as ONE batched
call (each window is its own sequence with its own length), not one call per window.

Batching (new, optional): ``inference`` takes per-sequence ``lengths``; row b's embedding is taken
at frame ``lengths[b] - 1`` and equals the reference run on ``x[b:b+1, :lengths[b]]``.
"""

from typing import Optional, Sequence

import numpy as np
import torch
from torch import nn

from ._lib import get_engine
from .params import host_tensors, new_token, populate
from .spec import Ge2eConfig, ge2e_spec

MAX_SEQS = 64  # sequences per library call


class SpeakerEncoder(nn.Module):
    def __init__(self, input_dim, proj_dim=256, lstm_dim=768, num_lstm_layers=3, use_lstm_with_projection=True):
        super().__init__()
        if lstm_dim != 768:
            raise NotImplementedError("lstm_dim must be 768 (the reference config; the HIP LSTM is built for it)")
        self.use_lstm_with_projection = use_lstm_with_projection
        self.cfg = Ge2eConfig(input_dim=input_dim, proj_dim=proj_dim, lstm_dim=lstm_dim,
                              num_lstm_layers=num_lstm_layers, use_lstm_with_projection=use_lstm_with_projection)
        populate(self, ge2e_spec(self.cfg))
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

    def forward(self, x):
        return self.inference(x)

    def _device(self):
        return next(self.parameters()).device

    def _sync(self, eng):
        key = (self._token, self._version)
        if eng.ge2e_key != key:
            c = self.cfg
            eng.load_ge2e(host_tensors(self), c.input_dim, c.proj_dim, c.lstm_dim, c.num_lstm_layers,
                          c.use_lstm_with_projection)
            eng.ge2e_key = key

    @torch.no_grad()
    def inference(self, x, lengths: Optional[Sequence[int]] = None):
        dev = self._device()
        eng = get_engine(dev)
        x = torch.as_tensor(x).to(dev, torch.float32)
        if x.dim() == 2:
            x = x[None]
        x = x.contiguous()
        B, T, D = x.shape
        if D != self.cfg.input_dim:
            raise ValueError(f"expected {self.cfg.input_dim} mel channels, got {D}")
        lens = np.full(B, T, np.int64) if lengths is None else np.asarray(torch.as_tensor(lengths).cpu(), np.int64)
        if len(lens) != B or lens.min() < 1 or lens.max() > T:
            raise ValueError("lengths must have B entries in [1, T]")
        out = torch.empty(B, self.cfg.proj_dim, device=dev)
        with eng.lock:
            self._sync(eng)
            for b0 in range(0, B, MAX_SEQS):
                b1 = min(B, b0 + MAX_SEQS)
                Tn = int(lens[b0:b1].max())
                eng.ge2e_infer(x[b0:b1, :Tn].contiguous(), lens[b0:b1], out[b0:b1])
        return out

    @torch.no_grad()
    def compute_embedding(self, x, num_frames=160, overlap=0.5):
        """Mean of the window embeddings of x (1 x T x D), windows as in model.py:70-88."""
        x = torch.as_tensor(x)
        if x.dim() == 2:
            x = x[None]
        num_overlap = int(num_frames * overlap)
        T = x.shape[1]
        starts = list(range(0, T, num_frames - num_overlap))
        wins = [(o, min(T, o + num_frames)) for o in starts]
        L = max(e - o for o, e in wins)
        batch = torch.zeros(len(wins), L, x.shape[2], dtype=torch.float32, device=x.device)
        for i, (o, e) in enumerate(wins):
            batch[i, :e - o] = x[0, o:e]
        emb = self.inference(batch, lengths=[e - o for o, e in wins])
        return (emb.sum(0, keepdim=True) / len(wins))
