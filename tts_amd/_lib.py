"""ctypes binding of ``libttship.so`` (the C ABI in ``include/ttship.h``).

The library is built in-tree (``tts_amd/libttship.so``, see ``tts_amd/csrc/Makefile`` and
``__graft_entry__.build``). There is no CPU fallback: if the library or a ROCm device is
missing, every entry point raises ``RuntimeError``.
"""

import atexit
import collections
import ctypes
import os
import threading
from typing import Dict

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TTSHIP_LIB", os.path.join(_HERE, "libttship.so"))

_lib = None
_lock = threading.Lock()

_c_int_p = ctypes.POINTER(ctypes.c_int32)
_c_i64_p = ctypes.POINTER(ctypes.c_int64)
_c_f_p = ctypes.POINTER(ctypes.c_float)
_c_i_p = ctypes.POINTER(ctypes.c_int)
_vp = ctypes.c_void_p

# (name, restype, argtypes) for every symbol declared in include/ttship.h
SIGNATURES = [
    ("tts_version", ctypes.c_int, []),
    ("tts_last_error", ctypes.c_char_p, []),
    ("tts_ctx_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    ("tts_ctx_destroy", ctypes.c_int, [_vp]),
    ("tts_taco_set_tensor", ctypes.c_int, [_vp, ctypes.c_char_p, _vp, _c_i64_p, ctypes.c_int]),
    ("tts_taco_finalize", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    ("tts_taco_infer", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_int_p,
                                      ctypes.c_int, ctypes.c_float, _vp, _vp, _vp, _vp, _c_int_p, _c_int_p, _vp]),
    ("tts_taco_infer_spk", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_int_p,
                                          ctypes.c_int, ctypes.c_float, _vp, _vp, _vp, _vp, _vp, _vp, _c_int_p,
                                          _c_int_p, _vp]),
    ("tts_taco_mbmelgan_infer", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               _c_int_p, ctypes.c_int, ctypes.c_float, _vp, _vp, _vp, _vp, _vp,
                                               _vp, ctypes.c_int, _vp, _c_int_p, _c_int_p, _vp]),
    ("tts_taco_mbmelgan_submit", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                _c_int_p, ctypes.c_int, ctypes.c_float, _vp, _vp, _vp, _vp, _vp,
                                                _vp, ctypes.c_int, _vp, _c_int_p, _c_int_p, _c_i64_p, _vp]),
    ("tts_taco_mbmelgan_finish", ctypes.c_int, [_vp, ctypes.c_int64, _vp]),
    ("tts_taco_speaker_dim", ctypes.c_int, [_vp, _c_i_p, _c_i_p]),
    ("tts_taco_set_options", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    ("tts_taco_encoder", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, _vp, _vp]),
    ("tts_taco_postnet", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, _vp, _vp]),
    ("tts_taco_decoder_state", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("tts_melgan_set_tensor", ctypes.c_int, [_vp, ctypes.c_char_p, _vp, _c_i64_p, ctypes.c_int]),
    ("tts_melgan_finalize", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_int_p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int]),
    ("tts_melgan_infer", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp]),
    ("tts_melgan_infer_strided", ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _c_int_p,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp]),
    ("tts_melgan_generator", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp,
                                            _vp]),
    ("tts_pqmf_synthesis", ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int,
                                          _vp, _vp]),
    ("tts_ge2e_set_tensor", ctypes.c_int, [_vp, ctypes.c_char_p, _vp, _c_i64_p, ctypes.c_int]),
    ("tts_ge2e_finalize", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int]),
    ("tts_ge2e_infer", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, _vp, _vp]),
    ("tts_pwgan_set_tensor", ctypes.c_int, [_vp, ctypes.c_char_p, _vp, _c_i64_p, ctypes.c_int]),
    ("tts_pwgan_finalize", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _c_int_p, ctypes.c_int]),
    ("tts_pwgan_infer", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp,
                                       _vp]),
    ("tts_glow_set_tensor", ctypes.c_int, [_vp, ctypes.c_char_p, _vp, _c_i64_p, ctypes.c_int]),
    ("tts_glow_finalize", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    ("tts_glow_encode", ctypes.c_int, [_vp, _vp, _c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, _c_int_p,
                                       _vp]),
    ("tts_glow_encode_spk", ctypes.c_int, [_vp, _vp, _c_int_p, _c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                           _c_int_p, _vp]),
    ("tts_glow_decode", ctypes.c_int, [_vp, _vp, ctypes.c_float, ctypes.c_int, _vp, _vp, _vp, _vp, _vp]),
    ("tts_time_decoder_kernel", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _c_f_p]),
    ("tts_decoder_stats", ctypes.c_int, [_vp, _c_i_p, _c_i_p, _c_f_p, _c_i_p]),
    ("tts_set_gemm_mode", ctypes.c_int, [_vp, ctypes.c_int]),
    ("tts_test_stall_lstm", ctypes.c_int, [ctypes.c_int]),
    ("tts_gemm_mode", ctypes.c_int, [_vp, _c_i_p, _c_i64_p]),
]


def load_library():
    """Load and type the shared library (no GPU calls are made here)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"libttship.so not found at {LIB_PATH}; run __graft_entry__.build() "
                                   f"(make -C tts_amd/csrc)")
            lib = ctypes.CDLL(LIB_PATH)
            for name, res, args in SIGNATURES:
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def _check(rc: int):
    if rc != 0:
        msg = load_library().tts_last_error()
        raise RuntimeError("ttship: " + (msg.decode() if msg else "unknown error"))


def _i32(a):
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.int32))
    return arr, arr.ctypes.data_as(_c_int_p)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream(device):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Engine:
    """One library context per device (owns packed weights, workspace, captured graphs)."""

    def __init__(self, device_index: int):
        self.lib = load_library()
        self.device = device_index
        # Held by every model across its weight check-and-upload (``_sync``) and its whole compute
        # sequence: the context's workspace, graphs and packed weights are shared by all models on
        # this device, and ctypes releases the GIL inside each call. (Each C entry point also locks
        # the context; this lock makes multi-call sequences such as Glow encode + decode atomic.)
        self.lock = threading.RLock()
        self._live = collections.OrderedDict()  # ticket -> (post, wav) of unfinished fused submissions
        h = ctypes.c_void_p()
        _check(self.lib.tts_ctx_create(device_index, ctypes.byref(h)))
        self.h = h
        self.taco_key = None
        self.melgan_key = None
        self.pwgan_key = None
        self.ge2e_key = None
        self.glow_key = None

    def close(self):
        if self.h:
            self.lib.tts_ctx_destroy(self.h)
            self.h = None

    # -- weights ---------------------------------------------------------------------
    def _set(self, fn, name, arr):
        a = np.ascontiguousarray(arr, dtype=np.float32)
        shape = (ctypes.c_int64 * max(1, a.ndim))(*a.shape)
        _check(fn(self.h, name.encode(), a.ctypes.data_as(ctypes.c_void_p), shape, a.ndim))

    def load_tacotron(self, tensors: Dict[str, np.ndarray], num_chars: int, r_init: int, attn_norm: str,
                      windowing: bool = False, forward_attn: bool = False, forward_attn_mask: bool = False):
        _check(self.lib.tts_taco_set_options(self.h, int(bool(windowing)), int(bool(forward_attn)),
                                             int(bool(forward_attn and forward_attn_mask))))
        for k, v in tensors.items():
            self._set(self.lib.tts_taco_set_tensor, k, v)
        _check(self.lib.tts_taco_finalize(self.h, num_chars, r_init, 1 if attn_norm == "softmax" else 0))

    def load_melgan(self, tensors: Dict[str, np.ndarray], in_channels, out_channels, base_channels,
                    upsample_factors, num_res_blocks, use_pqmf):
        for k, v in tensors.items():
            self._set(self.lib.tts_melgan_set_tensor, k, v)
        ups, ups_p = _i32(list(upsample_factors))
        _check(self.lib.tts_melgan_finalize(self.h, in_channels, out_channels, base_channels, ups_p, len(ups),
                                            num_res_blocks, 1 if use_pqmf else 0))

    # -- compute (device tensors) ----------------------------------------------------
    def taco_infer(self, ids, lens, r, max_steps, S_cap, stop_threshold, dec, post, align, stop,
                   speaker_ids=None, speaker_embeddings=None):
        B, T = ids.shape
        lens_a, lens_p = _i32(lens)
        ms_a, ms_p = _i32(max_steps)
        steps = np.zeros(B, np.int32)
        status = np.zeros(B, np.int32)
        if speaker_ids is None and speaker_embeddings is None:
            _check(self.lib.tts_taco_infer(self.h, _ptr(ids), lens_p, B, T, r, ms_p, S_cap, float(stop_threshold),
                                           _ptr(dec), _ptr(post), _ptr(align), _ptr(stop),
                                           steps.ctypes.data_as(_c_int_p), status.ctypes.data_as(_c_int_p),
                                           _stream(ids.device)))
        else:
            sid = None if speaker_ids is None else _ptr(speaker_ids)
            semb = None if speaker_embeddings is None else _ptr(speaker_embeddings)
            _check(self.lib.tts_taco_infer_spk(self.h, _ptr(ids), lens_p, B, T, r, ms_p, S_cap,
                                               float(stop_threshold), sid, semb, _ptr(dec), _ptr(post),
                                               _ptr(align), _ptr(stop), steps.ctypes.data_as(_c_int_p),
                                               status.ctypes.data_as(_c_int_p), _stream(ids.device)))
        return steps, status

    def taco_mbmelgan_infer(self, ids, lens, r, max_steps, S_cap, stop_threshold, dec, post, align, stop, pad, wav,
                            speaker_ids=None, speaker_embeddings=None):
        """Tacotron2 decode and MB-MelGAN on its postnet output in one library call
        (tts_taco_mbmelgan_infer); ``wav`` holds B * hop * (S_cap * r + 2 pad) floats."""
        B, T = ids.shape
        lens_a, lens_p = _i32(lens)
        ms_a, ms_p = _i32(max_steps)
        steps = np.zeros(B, np.int32)
        status = np.zeros(B, np.int32)
        sid = None if speaker_ids is None else _ptr(speaker_ids)
        semb = None if speaker_embeddings is None else _ptr(speaker_embeddings)
        _check(self.lib.tts_taco_mbmelgan_infer(self.h, _ptr(ids), lens_p, B, T, r, ms_p, S_cap, float(stop_threshold),
                                                sid, semb, _ptr(dec), _ptr(post), _ptr(align), _ptr(stop), int(pad),
                                                _ptr(wav), steps.ctypes.data_as(_c_int_p),
                                                status.ctypes.data_as(_c_int_p), _stream(ids.device)))
        return steps, status

    def taco_mbmelgan_submit(self, ids, lens, r, max_steps, S_cap, stop_threshold, dec, post, align, stop, pad, wav,
                             speaker_ids=None, speaker_embeddings=None):
        """The first half of taco_mbmelgan_infer (tts_taco_mbmelgan_submit): returns (steps, status,
        ticket) once the decode is done, the vocoder still running; ``post`` and ``wav`` must stay
        untouched until ``taco_mbmelgan_finish(ticket)``."""
        B, T = ids.shape
        lens_a, lens_p = _i32(lens)
        ms_a, ms_p = _i32(max_steps)
        steps = np.zeros(B, np.int32)
        status = np.zeros(B, np.int32)
        ticket = ctypes.c_int64(0)
        sid = None if speaker_ids is None else _ptr(speaker_ids)
        semb = None if speaker_embeddings is None else _ptr(speaker_embeddings)
        _check(self.lib.tts_taco_mbmelgan_submit(self.h, _ptr(ids), lens_p, B, T, r, ms_p, S_cap, float(stop_threshold),
                                                 sid, semb, _ptr(dec), _ptr(post), _ptr(align), _ptr(stop), int(pad),
                                                 _ptr(wav), steps.ctypes.data_as(_c_int_p),
                                                 status.ctypes.data_as(_c_int_p), ctypes.byref(ticket),
                                                 _stream(ids.device)))
        # a fp32 re-run at finish reads post and writes wav: keep them allocated while the library
        # may still do that (it finishes a ticket at the latest when the 5th submission after it
        # reuses its slot)
        self._live[ticket.value] = (post, wav)
        while len(self._live) > 4:
            self._live.popitem(last=False)
        return steps, status, ticket.value

    def taco_mbmelgan_finish(self, ticket, device):
        """Completes a submission (tts_taco_mbmelgan_finish): its waveforms are final after this."""
        _check(self.lib.tts_taco_mbmelgan_finish(self.h, int(ticket), _stream(device)))
        self._live.pop(int(ticket), None)

    def taco_speaker_dim(self):
        d, n = ctypes.c_int(0), ctypes.c_int(0)
        _check(self.lib.tts_taco_speaker_dim(self.h, ctypes.byref(d), ctypes.byref(n)))
        return d.value, n.value

    def taco_encoder(self, ids, lens, out):
        B, T = ids.shape
        lens_a, lens_p = _i32(lens)
        _check(self.lib.tts_taco_encoder(self.h, _ptr(ids), lens_p, B, T, _ptr(out), _stream(ids.device)))

    def taco_postnet(self, dec, lens, out):
        B, M, _ = dec.shape
        lens_a, lens_p = _i32(lens)
        _check(self.lib.tts_taco_postnet(self.h, _ptr(dec), lens_p, B, M, _ptr(out), _stream(dec.device)))

    def taco_decoder_state(self, B, T_max, device, key=None):
        """Decoder state after the last Tacotron2 decode (tts_taco_decoder_state), caller row order.
        ``key``: the calling model's weight key; the read is refused if another model (or another
        version of this one) decoded on this device since."""
        import torch
        out = {k: torch.empty(B, n, device=device) for k, n in
               (("query", 1024), ("attention_rnn_cell_state", 1024), ("decoder_hidden", 1024),
                ("decoder_cell", 1024), ("context", 512), ("attention_weights", T_max),
                ("attention_weights_cum", T_max))}
        with self.lock:
            if key is not None and self.taco_key != key:
                raise RuntimeError("decoder_state: another Tacotron2 model decoded on this device since this model's call")
            _check(self.lib.tts_taco_decoder_state(self.h, B, T_max, *[_ptr(out[k]) for k in out], _stream(device)))
        return out

    def load_pwgan(self, tensors: Dict[str, np.ndarray], num_res_blocks, stacks, upsample_factors):
        for k, v in tensors.items():
            self._set(self.lib.tts_pwgan_set_tensor, k, v)
        ups, ups_p = _i32(list(upsample_factors))
        _check(self.lib.tts_pwgan_finalize(self.h, num_res_blocks, stacks, ups_p, len(ups)))

    def pwgan_infer(self, mel, lens, pad, noise, out):
        B, _, M = mel.shape
        lens_a, lens_p = _i32(lens)
        _check(self.lib.tts_pwgan_infer(self.h, _ptr(mel), lens_p, B, M, pad, _ptr(noise), _ptr(out),
                                        _stream(mel.device)))

    def load_glow(self, tensors: Dict[str, np.ndarray], num_chars, enc_layers, flows, wn_layers):
        for k, v in tensors.items():
            self._set(self.lib.tts_glow_set_tensor, k, v)
        _check(self.lib.tts_glow_finalize(self.h, num_chars, enc_layers, flows, wn_layers))

    def glow_encode(self, ids, lens, length_scale, speaker_ids=None):
        B, T = ids.shape
        lens_a, lens_p = _i32(lens)
        ylens = np.zeros(B, np.int32)
        if speaker_ids is None:
            _check(self.lib.tts_glow_encode(self.h, _ptr(ids), lens_p, B, T, float(length_scale),
                                            ylens.ctypes.data_as(_c_int_p), _stream(ids.device)))
        else:
            spk_a, spk_p = _i32(speaker_ids)
            if len(spk_a) != B:
                raise ValueError("one speaker id per utterance")
            _check(self.lib.tts_glow_encode_spk(self.h, _ptr(ids), lens_p, spk_p, B, T, float(length_scale),
                                                ylens.ctypes.data_as(_c_int_p), _stream(ids.device)))
        return ylens

    def glow_decode(self, noise, noise_scale, Ty, y, y_mean, attn, logw):
        _check(self.lib.tts_glow_decode(self.h, _ptr(noise), float(noise_scale), Ty, _ptr(y), _ptr(y_mean),
                                        _ptr(attn), _ptr(logw), _stream(y.device)))

    def load_ge2e(self, tensors: Dict[str, np.ndarray], input_dim, proj_dim, lstm_dim, num_layers, with_proj):
        for k, v in tensors.items():
            self._set(self.lib.tts_ge2e_set_tensor, k, v)
        _check(self.lib.tts_ge2e_finalize(self.h, input_dim, proj_dim, lstm_dim, num_layers, 1 if with_proj else 0))

    def ge2e_infer(self, x, lens, out):
        B, T, _ = x.shape
        lens_a, lens_p = _i32(lens)
        _check(self.lib.tts_ge2e_infer(self.h, _ptr(x), lens_p, B, T, _ptr(out), _stream(x.device)))

    def melgan_infer(self, mel, lens, pad, wav):
        """mel (B, C, M): contiguous, or any strided view the library reads in place (e.g. a
        (B, M, C) postnet output transposed)."""
        B, _, M = mel.shape
        lens_a, lens_p = _i32(lens)
        if mel.is_contiguous():
            _check(self.lib.tts_melgan_infer(self.h, _ptr(mel), lens_p, B, M, pad, _ptr(wav), _stream(mel.device)))
        else:
            sb, sc, st = mel.stride()
            _check(self.lib.tts_melgan_infer_strided(self.h, _ptr(mel), sb, sc, st, lens_p, B, M, pad, _ptr(wav),
                                                     _stream(mel.device)))

    def melgan_generator(self, mel, lens, pad, out):
        B, _, M = mel.shape
        lens_a, lens_p = _i32(lens)
        _check(self.lib.tts_melgan_generator(self.h, _ptr(mel), lens_p, B, M, pad, _ptr(out),
                                             _stream(mel.device)))

    def pqmf_synthesis(self, x, G, y):
        B, N, L = x.shape
        taps = G.shape[-1] - 1
        _check(self.lib.tts_pqmf_synthesis(self.h, _ptr(x), B, N, L, _ptr(G), taps, _ptr(y), _stream(x.device)))

    def decoder_stats(self):
        """(path, [(ms, steps) per persistent launch]) of the last Tacotron2 decode."""
        path, n = ctypes.c_int(0), ctypes.c_int(0)
        ms = (ctypes.c_float * 4)()   # up to 4 persistent launches (batch tiles of 64, 48, 32, 16 rows)
        st = (ctypes.c_int * 4)()
        _check(self.lib.tts_decoder_stats(self.h, ctypes.byref(path), ctypes.byref(n), ms, st))
        return int(path.value), [(float(ms[i]), int(st[i])) for i in range(n.value)]

    def set_gemm_mode(self, mode: str):
        """'x3' = split-f16 MFMA GEMMs where built (fp32-accurate, the default), 'f32' = fp32 MFMA."""
        if mode not in ("x3", "f32"):
            raise ValueError("gemm mode must be 'x3' or 'f32'")
        with self.lock:
            _check(self.lib.tts_set_gemm_mode(self.h, 1 if mode == "x3" else 0))

    def gemm_mode(self):
        """(mode, calls re-run in fp32 because an operand left the f16 range)."""
        m, n = ctypes.c_int(0), ctypes.c_int64(0)
        _check(self.lib.tts_gemm_mode(self.h, ctypes.byref(m), ctypes.byref(n)))
        return ("x3" if m.value else "f32"), int(n.value)

    def time_decoder_kernel(self, which: int, iters: int) -> float:
        ms = ctypes.c_float(0.0)
        _check(self.lib.tts_time_decoder_kernel(self.h, which, iters, ctypes.byref(ms)))
        return float(ms.value)


_engines: Dict[int, Engine] = {}


def get_engine(device) -> Engine:
    """Engine for a torch device (must be a ROCm 'cuda' device)."""
    import torch
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError("tts_amd runs on MI355X (ROCm 'cuda' devices) only; got device "
                           f"'{dev}'. There is no CPU fallback: move the model with .cuda().")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    with _lock:
        eng = _engines.get(idx)
    if eng is None:
        eng = Engine(idx)
        with _lock:
            _engines[idx] = eng
    return eng


@atexit.register
def _close_engines():
    """Destroy every context (graphs, streams, device buffers) before interpreter teardown, so the
    HIP runtime and any attached tool (rocprofv3) never see leaked objects after finalisation."""
    with _lock:
        engines = list(_engines.values())
        _engines.clear()
    for eng in engines:
        try:
            eng.close()
        except Exception:
            pass
