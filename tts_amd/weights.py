"""Version-stable synthetic weights (no torch / numpy RNG streams involved).

No trained checkpoint exists offline, so parity fixtures, tests and the
benchmark all use weights from this generator: a splitmix64 counter stream keyed by
``(seed, fnv1a64(parameter name))``, mapped to uniform [-1, 1) and scaled per tensor kind
with xavier-like / PyTorch-default-like bounds (``TTS/tts/layers/common_layers.py:17-20``
uses xavier_uniform; ``nn.LSTMCell`` uses U(-1/sqrt(H), 1/sqrt(H))). The same seed gives
bit-identical float32 weights on every machine, so fixtures store only the seed.
"""

import math
from typing import Dict, Iterable, Optional, Tuple

import numpy as np

_M64 = (1 << 64) - 1


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & _M64
    return h


def splitmix64_uniform(key: int, n: int) -> np.ndarray:
    """n float64 values uniform in [-1, 1) from the splitmix64 stream at ``key``."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(key & _M64) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))
    return 2.0 * u - 1.0


_GAIN = {"linear": 1.0, "linear_relu": math.sqrt(2.0), "linear_tanh": 5.0 / 3.0,
         "linear_sigmoid": 1.0, "attn_v": 1.0}


def _fans(shape: Tuple[int, ...]) -> Tuple[int, int]:
    if len(shape) < 2:
        return shape[0], shape[0]
    rf = int(np.prod(shape[2:])) if len(shape) > 2 else 1
    return shape[1] * rf, shape[0] * rf


def synth_tensor(name: str, shape: Tuple[int, ...], kind: str, seed: int,
                 overrides: Optional[Dict[str, float]] = None) -> np.ndarray:
    """Deterministic float32 tensor for one parameter."""
    n = int(np.prod(shape)) if len(shape) else 1
    if kind == "count":
        return np.zeros(shape, dtype=np.int64)
    if kind == "buffer":
        raise ValueError("buffers are computed, not sampled: " + name)
    u = splitmix64_uniform((seed * 0x9E3779B97F4A7C15 + fnv1a64(name)) & _M64, n)
    sc = (overrides or {}).get(kind)
    if kind == "embedding":
        a = math.sqrt(6.0 / (shape[0] + shape[1]))
        x = u * a
    elif kind in _GAIN:
        fi, fo = _fans(shape)
        a = _GAIN[kind] * math.sqrt(6.0 / (fi + fo))
        x = u * a
    elif kind == "conv":
        fi, fo = _fans(shape)
        x = u * math.sqrt(6.0 / (fi + fo))
    elif kind in ("lstm", "lstm_enc"):
        H = shape[0] // 4
        x = u / math.sqrt(H)
    elif kind == "xavier":  # xavier_normal_ in the reference (speaker_encoder/model.py:49-54): same std
        fi, fo = _fans(shape)
        x = u * math.sqrt(3.0) * math.sqrt(2.0 / (fi + fo))
    elif kind == "glow_emb":  # normal_(0, hidden ** -0.5) (glow_tts/encoder.py:61): same std
        x = u * math.sqrt(3.0) * shape[1] ** -0.5
    elif kind == "dwconv":  # depthwise conv (groups = channels): fan_in = taps, kaiming-uniform scale
        x = u * math.sqrt(1.0 / shape[-1])
    elif kind == "ln_g":
        x = 1.0 + 0.1 * u
    elif kind == "actnorm":
        x = 0.05 * u
    elif kind == "glow_end":  # zero-initialised in the reference; small so the flows stay tame
        fi, fo = _fans(shape)
        x = 0.1 * u * math.sqrt(6.0 / (fi + fo))
    elif kind == "orthogonal":  # a rotation (QR of a splitmix64 matrix), det > 0 as in glow.py:172-175
        q, r = np.linalg.qr(u.reshape(shape))
        q = q * np.sign(np.diag(r))[None, :]
        if np.linalg.det(q) < 0:
            q[:, 0] = -q[:, 0]
        x = q.reshape(-1)
    elif kind == "glow_spk":  # uniform_(-0.1, 0.1) (glow_tts.py:98-99)
        x = 0.1 * u
    elif kind == "speaker_emb":  # normal_(0, 0.3) in the reference: same std, uniform
        x = u * (0.3 * math.sqrt(3.0))
    elif kind == "bias":
        x = 0.05 * u
    elif kind == "stop_bias":
        x = np.full(n, 0.0)
    elif kind == "bn_w":
        x = 1.0 + 0.1 * u
    elif kind == "bn_b":
        x = 0.05 * u
    elif kind == "bn_mean":
        x = 0.05 * u
    elif kind == "bn_var":
        x = 1.0 + 0.25 * (u + 1.0)
    elif kind == "wn_g":
        x = 1.0 + 0.1 * u
    else:
        raise ValueError(f"unknown kind {kind} for {name}")
    if sc is not None:
        x = x * sc
    return x.astype(np.float32).reshape(shape)


def synth_state_dict(spec: Iterable[Tuple[str, Tuple[int, ...], str]], seed: int,
                     overrides: Optional[Dict[str, float]] = None,
                     skip_buffers: bool = True) -> Dict[str, np.ndarray]:
    out = {}
    for name, shape, kind in spec:
        if kind == "buffer":
            if skip_buffers:
                continue
        out[name] = synth_tensor(name, tuple(shape), kind, seed, overrides)
    return out
