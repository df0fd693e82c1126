"""Drop-in ``Tacotron2`` whose ``inference`` runs on MI355X through ``libttship.so``.

Mirrors the reference surface used by ``TTS/server/synthesizer.py:43-79`` and
``TTS/tts/utils/synthesis.py:48-67``: the constructor signature of
``TTS/tts/models/tacotron2.py:10-37``, checkpoint keys (``load_state_dict(cp['model'])``),
``.cuda()`` / ``.eval()``, ``decoder.set_r(r)`` (``layers/tacotron2.py:208-209``),
``decoder.max_decoder_steps`` (``:156``) and ``inference(text, speaker_ids, style_mel,
speaker_embeddings)`` returning ``(decoder_outputs (B,M,80), postnet_outputs (B,M,80),
alignments (B,S,T), stop_tokens (B,S,1))`` (``models/tacotron2.py:142-163``).

Batching (new, optional): ``text`` may hold B > 1 padded rows with ``text_lengths``; row i
of the outputs equals the reference B=1 call on utterance i (the reference itself cannot
run B > 1: ``layers/tacotron2.py:362``). Per-utterance lengths are in ``last_steps`` /
``last_mel_lengths`` after the call; padded positions are zero.
"""

from typing import Optional, Sequence

import numpy as np
import torch
from torch import nn

from ._lib import get_engine
from .params import Container, host_tensors, new_token, populate
from .spec import TacotronConfig, tacotron2_spec

BATCH_LIMIT = 64
SPEAKER_BATCH_LIMIT = 64  # multi-speaker / decoder variants run on the persistent decoder (<= 64 rows)


class Decoder(Container):
    """Holds decoder parameters plus the runtime knobs the reference exposes."""

    def __init__(self, r: int, frame_channels: int = 80):
        super().__init__()
        self.r_init = r
        self.r = r
        self.frame_channels = frame_channels
        self.max_decoder_steps = 1000
        self.stop_threshold = 0.5

    def set_r(self, new_r):
        self.r = int(new_r)


class VocodedResult:
    """A submitted ``Tacotron2.inference_vocoded_submit`` call. ``outputs`` holds the decode's
    (decoder_outputs, postnet_outputs, alignments, stop_tokens), ready on return; the waveforms are
    final once ``result()`` has returned (it completes the library ticket)."""

    def __init__(self, outputs, wav, eng=None, ticket=None):
        self.outputs = outputs
        self._wav = wav
        self._eng, self._ticket = eng, ticket

    def result(self):
        if self._ticket is not None:
            with self._eng.lock:
                self._eng.taco_mbmelgan_finish(self._ticket, self._wav.device)
            self._ticket = None
        return tuple(self.outputs) + (self._wav,)


class Tacotron2(nn.Module):
    def __init__(self, num_chars, num_speakers=0, r=7, postnet_output_dim=80, decoder_output_dim=80,
                 attn_type="original", attn_win=False, attn_norm="softmax", prenet_type="original",
                 prenet_dropout=True, forward_attn=False, trans_agent=False, forward_attn_mask=False,
                 location_attn=True, attn_K=5, separate_stopnet=True, bidirectional_decoder=False,
                 double_decoder_consistency=False, ddc_r=None, encoder_in_features=512,
                 decoder_in_features=512, speaker_embedding_dim=None, gst=False, gst_embedding_dim=512,
                 gst_num_heads=4, gst_style_tokens=10, gst_use_speaker_embedding=False):
        super().__init__()
        unsupported = []
        if gst:
            unsupported.append("GST")
        if attn_type not in ("original", "graves"):
            unsupported.append(f"attn_type={attn_type}")
        if trans_agent and not forward_attn:
            unsupported.append("trans_agent without forward_attn")
        if not location_attn:
            unsupported.append("location_attn=False")
        if prenet_type not in ("original", "bn"):
            unsupported.append(f"prenet_type={prenet_type}")
        if encoder_in_features != 512 or decoder_in_features != 512:  # before the speaker columns
            unsupported.append("non-default encoder/decoder feature sizes")
        if decoder_output_dim != 80 or postnet_output_dim != 80:
            unsupported.append("frame channels != 80")
        if attn_norm not in ("sigmoid", "softmax"):
            raise ValueError("Unknown value for attention norm type")
        if unsupported:
            raise NotImplementedError("tts_amd Tacotron2 does not implement: " + ", ".join(unsupported) +
                                      " (SURVEY.md §8f lists these as next steps)")
        self.num_chars = num_chars
        self.num_speakers = num_speakers
        self.r = r
        self.attn_norm = attn_norm
        self.double_decoder_consistency = double_decoder_consistency
        self.cfg = TacotronConfig(num_chars=num_chars, r=r, attn_norm=attn_norm,
                                  double_decoder_consistency=double_decoder_consistency,
                                  ddc_r=ddc_r if ddc_r is not None else r,
                                  num_speakers=num_speakers, speaker_embedding_dim=speaker_embedding_dim,
                                  prenet_type=prenet_type, attn_type=attn_type, attn_K=attn_K,
                                  bidirectional_decoder=bool(bidirectional_decoder),
                                  # GravesAttention ignores the location-attention options (tacotron2.py:177-188)
                                  windowing=bool(attn_win) and attn_type != "graves",
                                  forward_attn=bool(forward_attn) and attn_type != "graves",
                                  trans_agent=bool(trans_agent) and attn_type != "graves",
                                  forward_attn_mask=bool(forward_attn and forward_attn_mask) and attn_type != "graves")
        # models/tacotron2.py:50-58 / tacotron_abstract.py:76-81: a learned table unless the caller
        # gives per-sample embeddings of speaker_embedding_dim
        self.embeddings_per_sample = speaker_embedding_dim is not None
        self.speaker_embedding_dim = self.cfg.spk_dim
        self.decoder = Decoder(r, decoder_output_dim)
        populate(self, tacotron2_spec(self.cfg))
        self._version = 0
        self._token = new_token()
        self.last_steps = None
        self.last_mel_lengths = None
        self.last_status = None

    def _speaker_args(self, speaker_ids, speaker_embeddings, B, dev):
        """Speaker conditioning as the reference takes it (models/tacotron2.py:152-155): ids into
        the learned table, or per-sample embeddings (B, speaker_embedding_dim) / (B, 1, dim)."""
        if self.num_speakers <= 1:  # the reference ignores both arguments here (models/tacotron2.py:152)
            return None, None
        if self.embeddings_per_sample:
            if speaker_embeddings is None:
                raise ValueError("this model takes per-sample speaker_embeddings")
            e = torch.as_tensor(speaker_embeddings).to(dev, torch.float32).reshape(-1, self.speaker_embedding_dim)
            if e.shape[0] == 1 and B > 1:
                e = e.expand(B, -1)
            if e.shape[0] != B:
                raise ValueError("speaker_embeddings must have one row per utterance")
            return None, e.contiguous()
        if speaker_ids is None:
            raise ValueError("multi-speaker model: speaker_ids are required")
        ids = torch.as_tensor(speaker_ids).reshape(-1).to(torch.int64)
        if ids.numel() == 1 and B > 1:
            ids = ids.expand(B)
        if ids.numel() != B:
            raise ValueError("speaker_ids must have one entry per utterance")
        if int(ids.min()) < 0 or int(ids.max()) >= self.num_speakers:
            raise IndexError("speaker id out of range")  # nn.Embedding raises too
        return ids.to(dev).contiguous(), None

    # any change of parameters or placement invalidates the packed device copy
    def load_state_dict(self, state_dict, strict=True, **kw):
        res = super().load_state_dict(state_dict, strict=strict, **kw)
        self._version += 1
        return res

    def _apply(self, fn, *args, **kwargs):
        res = super()._apply(fn, *args, **kwargs)
        self._version += 1
        return res

    def invalidate(self):
        """Call after editing parameters in place."""
        self._version += 1

    def forward(self, *args, **kwargs):
        raise NotImplementedError("training forward is out of scope; use inference()")

    def _sync(self, eng):
        key = (self._token, self._version)
        if eng.taco_key != key:
            eng.load_tacotron(host_tensors(self, skip_prefixes=("coarse_decoder.", "decoder_backward.")), self.num_chars,
                              self.decoder.r_init, self.attn_norm, self.cfg.windowing, self.cfg.forward_attn,
                              self.cfg.forward_attn_mask)
            eng.taco_key = key

    def _prepare(self, text, speaker_ids, speaker_embeddings, text_lengths, max_decoder_steps):
        """Arguments of one inference call, checked and placed: (device, engine, ids, lengths, per-row
        max steps, r, speaker ids / embeddings, rows per library call)."""
        dev = self.embedding.weight.device
        eng = get_engine(dev)
        text = torch.as_tensor(text).to(dev, torch.int64)
        if text.dim() == 1:
            text = text[None]
        text = text.contiguous()
        B, T = text.shape
        lens = np.full(B, T, np.int64) if text_lengths is None else np.asarray(
            torch.as_tensor(text_lengths).cpu(), dtype=np.int64)
        if len(lens) != B or lens.min() < 1 or lens.max() > T:
            raise ValueError("text_lengths must have B entries in [1, T]")
        ms = self.decoder.max_decoder_steps if max_decoder_steps is None else max_decoder_steps
        ms = np.broadcast_to(np.asarray(ms, dtype=np.int64), (B,)).copy()
        r = int(self.decoder.r)
        if not 1 <= r <= self.decoder.r_init:
            raise ValueError(f"r={r} must be in [1, r_init={self.decoder.r_init}]")
        spk_ids, spk_emb = self._speaker_args(speaker_ids, speaker_embeddings, B, dev)
        variant = self.cfg.prenet_type == "bn" or self.cfg.windowing or self.cfg.forward_attn or \
            self.cfg.attn_type == "graves"
        limit = BATCH_LIMIT if self.num_speakers <= 1 and not variant else SPEAKER_BATCH_LIMIT
        return dev, eng, text, lens, ms, r, spk_ids, spk_emb, limit

    @staticmethod
    def _out_tensors(nb, S_cap, r, Tn, dev):
        dec = torch.empty(nb, S_cap * r, 80, device=dev, dtype=torch.float32)
        return (dec, torch.empty_like(dec), torch.empty(nb, S_cap, Tn, device=dev, dtype=torch.float32),
                torch.empty(nb, S_cap, device=dev, dtype=torch.float32))

    @torch.no_grad()
    def inference(self, text, speaker_ids=None, style_mel=None, speaker_embeddings=None,
                  text_lengths: Optional[Sequence[int]] = None, max_decoder_steps=None):
        if style_mel is not None:
            raise NotImplementedError("GST style conditioning is not implemented (SURVEY.md §8f)")
        dev, eng, text, lens, ms, r, spk_ids, spk_emb, limit = self._prepare(
            text, speaker_ids, speaker_embeddings, text_lengths, max_decoder_steps)
        B = text.shape[0]
        outs = []
        with eng.lock:
            self._sync(eng)
            for b0 in range(0, B, limit):
                b1 = min(B, b0 + limit)
                Tn = int(lens[b0:b1].max())
                sub = text[b0:b1, :Tn].contiguous()
                S_cap = int(ms[b0:b1].max())
                dec, post, align, stop = self._out_tensors(b1 - b0, S_cap, r, Tn, dev)
                steps, status = eng.taco_infer(
                    sub, lens[b0:b1], r, ms[b0:b1], S_cap, self.decoder.stop_threshold, dec, post, align, stop,
                    speaker_ids=None if spk_ids is None else spk_ids[b0:b1].contiguous(),
                    speaker_embeddings=None if spk_emb is None else spk_emb[b0:b1].contiguous())
                outs.append((dec, post, align, stop, steps, status))
        return self._assemble(outs, text.shape, lens, r, dev)

    def _assemble(self, outs, shape, lens, r, dev):
        """The library calls' outputs as the reference's (B, M, 80) x 2, (B, S, T), (B, S, 1), and the
        per-row lengths on ``self`` (last_steps, last_mel_lengths, last_status)."""
        B, T = shape
        steps = np.concatenate([o[4] for o in outs])
        status = np.concatenate([o[5] for o in outs])
        if getattr(self.decoder, "verbose", True):  # reference behaviour (tacotron2.py:365); bench.py mutes it
            for s in status:
                if s == 2:
                    print("   | > Decoder stopped with 'max_decoder_steps")
        S = int(steps.max())
        M = S * r
        if len(outs) == 1:
            dec, post, align, stop = outs[0][0][:, :M], outs[0][1][:, :M], outs[0][2][:, :S], outs[0][3][:, :S]
            if align.shape[2] != T:
                align = torch.nn.functional.pad(align, (0, T - align.shape[2]))
        else:
            # chunks of a split batch decode to their own S_cap; each is cut or zero-padded to the
            # batch's S steps (M frames) before joining (a chunk's rows are zero past their own steps)
            dec = torch.zeros(B, M, 80, device=dev)
            post = torch.zeros(B, M, 80, device=dev)
            align = torch.zeros(B, S, T, device=dev)
            stop = torch.zeros(B, S, device=dev)
            b0 = 0
            for o in outs:
                n, Sc, Tn = o[2].shape
                s_ = min(S, Sc)
                dec[b0:b0 + n, :s_ * r] = o[0][:, :s_ * r]
                post[b0:b0 + n, :s_ * r] = o[1][:, :s_ * r]
                align[b0:b0 + n, :s_, :Tn] = o[2][:, :s_]
                stop[b0:b0 + n, :s_] = o[3][:, :s_]
                b0 += n
        self.last_steps = steps
        self.last_mel_lengths = steps * r
        self.last_status = status
        self._last_call = (B, int(lens.max()), len(outs))
        return dec, post, align, stop[:, :, None]

    @torch.no_grad()
    def inference_vocoded(self, text, vocoder, speaker_ids=None, speaker_embeddings=None,
                          text_lengths: Optional[Sequence[int]] = None, max_decoder_steps=None):
        """``inference`` followed by ``vocoder.inference(postnet_outputs.transpose(1, 2),
        lengths=last_mel_lengths)`` -- the pair TTS/server/synthesizer.py:150-159 runs -- in one
        library call when ``vocoder`` is a MultibandMelganGenerator on the same device and the batch
        fits one decode (tts_taco_mbmelgan_infer: the vocoder is launched on the decoded lengths the
        decode leaves on the device, no host round trip between the models); otherwise the two
        calls. Returns (decoder_outputs, postnet_outputs, alignments, stop_tokens, waveforms (B, 1,
        hop * (M + 2 pad))), bit-identical to the two calls either way."""
        return self._vocoded(text, vocoder, speaker_ids, speaker_embeddings, text_lengths, max_decoder_steps,
                             submit=False).result()

    @torch.no_grad()
    def inference_vocoded_submit(self, text, vocoder, speaker_ids=None, speaker_embeddings=None,
                                 text_lengths: Optional[Sequence[int]] = None, max_decoder_steps=None):
        """``inference_vocoded`` in two halves (tts_taco_mbmelgan_submit / _finish): returns a
        ``VocodedResult`` once the decode is done, with the vocoder still running on the device, so
        that the caller can queue the next batch behind it; ``.result()`` waits for the vocoder
        (re-running it in fp32 if its split-f16 operands left the f16 range) and returns what
        ``inference_vocoded`` returns. The decode outputs (``.outputs[:4]``) are ready at once."""
        return self._vocoded(text, vocoder, speaker_ids, speaker_embeddings, text_lengths, max_decoder_steps,
                             submit=True)

    def _vocoded(self, text, vocoder, speaker_ids, speaker_embeddings, text_lengths, max_decoder_steps, submit):
        from .vocoder import MultibandMelganGenerator
        dev, eng, text, lens, ms, r, spk_ids, spk_emb, limit = self._prepare(
            text, speaker_ids, speaker_embeddings, text_lengths, max_decoder_steps)
        B = text.shape[0]
        vdev = vocoder.layers._modules["1"].bias.device if isinstance(vocoder, MultibandMelganGenerator) else None
        if vdev != dev or B > limit or vocoder.cfg.in_channels != 80:
            dec, post, align, stop = self.inference(text, speaker_ids=speaker_ids, speaker_embeddings=speaker_embeddings,
                                                    text_lengths=lens, max_decoder_steps=ms)
            wav = vocoder.inference(post.transpose(1, 2), lengths=self.last_mel_lengths)
            return VocodedResult((dec, post, align, stop), wav)
        pad = int(vocoder.inference_padding)
        Tn = int(lens.max())
        sub = text[:, :Tn].contiguous()
        S_cap = int(ms.max())
        dec, post, align, stop = self._out_tensors(B, S_cap, r, Tn, dev)
        hop = vocoder.hop
        wbuf = torch.empty(B * hop * (S_cap * r + 2 * pad), device=dev, dtype=torch.float32)
        with eng.lock:
            self._sync(eng)
            vocoder._sync(eng)
            args = (sub, lens, r, ms, S_cap, self.decoder.stop_threshold, dec, post, align, stop, pad, wbuf)
            if submit:
                steps, status, ticket = eng.taco_mbmelgan_submit(*args, speaker_ids=spk_ids, speaker_embeddings=spk_emb)
            else:
                steps, status = eng.taco_mbmelgan_infer(*args, speaker_ids=spk_ids, speaker_embeddings=spk_emb)
                ticket = None
        res = self._assemble([(dec, post, align, stop, steps, status)], text.shape, lens, r, dev)
        L = hop * (int(steps.max()) * r + 2 * pad)
        return VocodedResult(res, wbuf[:B * L].view(B, 1, L), eng, ticket)

    @torch.no_grad()
    def decoder_state(self):
        """The decoder state the reference leaves on ``self.decoder`` after ``inference`` (query,
        attention_rnn_cell_state, decoder_hidden, decoder_cell, context,
        attention.attention_weights / attention_weights_cum; layers/tacotron2.py:217-233,259-298,
        common_layers.py:251-260), for the last call's rows in caller order: (B, 1024) x 4,
        (B, 512), (B, T) x 2. Rows that stopped before the call's last step hold the batched
        decode's state, not their own final one (the reference decodes B = 1)."""
        B, T, nchunks = getattr(self, "_last_call", (0, 0, 0))
        if not B:
            raise RuntimeError("run inference first")
        if nchunks != 1:
            raise RuntimeError("decoder_state: the last call was split into several library calls")
        dev = self.embedding.weight.device
        eng = get_engine(dev)
        st = eng.taco_decoder_state(B, T, dev, key=(self._token, self._version))
        return st
