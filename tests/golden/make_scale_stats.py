"""Writes tests/golden/scale_stats_ref.npz from the reference's own mean-var stats fixture
(`tests/inputs/scale_stats.npy`, used by the reference's `tests/test_audio.py:157-176`), plus the
audio section of its `tests/inputs/test_config.json` and the samples of `tests/inputs/example_1.wav`
that test uses. Run in the build container (the reference is not on the GPU box):

    python tests/golden/make_scale_stats.py

The stats file is a pickled dict (`np.save(path, stats_dict)`, `TTS/bin/compute_statistics.py:80`).
No unpickler runs on it: the pickle stream is walked statically with `pickletools.genops` (a
disassembler: it yields opcodes and their arguments and executes nothing), and the values are
rebuilt from the opcode arguments alone. Only the opcodes numpy's array pickles and a dict of
scalars use are accepted; a GLOBAL is recorded as a name, never imported, and the only "call" the
walker understands is numpy's `_reconstruct` / `dtype` pattern, whose raw bytes and dtype string it
reads from the BUILD state.
"""
import json
import os
import pickletools
import sys
import wave

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


class _Call:
    """A REDUCE left unevaluated: the callable's dotted name and its arguments."""

    def __init__(self, fn, args):
        self.fn, self.args, self.state = fn, args, None


def static_stats(path):
    with open(path, "rb") as f:
        version = np.lib.format.read_magic(f)
        (np.lib.format.read_array_header_1_0 if version == (1, 0) else np.lib.format.read_array_header_2_0)(f)
        data = f.read()
    stack, memo, marks = [], {}, []
    for op, arg, _ in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "GLOBAL":
            stack.append(arg.replace(" ", "."))
        elif n in ("BINUNICODE", "SHORT_BINUNICODE", "BININT", "BININT1", "BININT2", "BINFLOAT",
                   "BINBYTES", "SHORT_BINBYTES"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n in ("NEWTRUE", "NEWFALSE"):
            stack.append(n == "NEWTRUE")
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            stack[-k:] = [tuple(stack[-k:])]
        elif n == "MARK":
            marks.append(len(stack))
        elif n == "TUPLE":
            m = marks.pop()
            stack[m:] = [tuple(stack[m:])]
        elif n in ("EMPTY_DICT", "EMPTY_LIST"):
            stack.append({} if n == "EMPTY_DICT" else [])
        elif n == "SETITEMS":
            m = marks.pop()
            items = stack[m:]
            del stack[m:]
            for k in range(0, len(items), 2):
                stack[-1][items[k]] = items[k + 1]
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "APPENDS":
            m = marks.pop()
            items = stack[m:]
            del stack[m:]
            stack[-1].extend(items)
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n in ("BINPUT", "LONG_BINPUT"):
            memo[arg] = stack[-1]
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif n == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            if fn not in ("numpy.core.multiarray._reconstruct", "numpy.dtype"):
                raise ValueError(f"{path}: unexpected callable {fn}")
            stack.append(_Call(fn, args))
        elif n == "BUILD":
            state = stack.pop()
            stack[-1].state = state
        elif n == "STOP":
            break
        else:
            raise ValueError(f"{path}: opcode {n} not handled by the static walker")
    root = stack[-1]

    def value(v):
        if isinstance(v, _Call) and v.fn == "numpy.core.multiarray._reconstruct":
            _, shape, dt, fortran, raw = v.state
            if isinstance(raw, _Call) or isinstance(raw, list):
                raise ValueError("object arrays other than the outer container are not expected")
            code = dt.args[0]
            order = dt.state[1]
            arr = np.frombuffer(raw, dtype=np.dtype(order + code if order in "<>" else code)).reshape(shape)
            return arr.copy(order="F" if fortran else "C")
        if isinstance(v, dict):
            return {k: value(x) for k, x in v.items()}
        return v

    # the outer 0-d object array holds the dict as its single element (BUILD state's last entry)
    outer = root.state[-1]
    items = outer[0] if isinstance(outer, list) else outer
    return value(items)


def main():
    sys.path.insert(0, ROOT)
    from tts_amd.factories import load_config
    stats = static_stats(os.path.join(REF, "tests", "inputs", "scale_stats.npy"))
    conf = load_config(os.path.join(REF, "tests", "inputs", "test_config.json"))
    with wave.open(os.path.join(REF, "tests", "inputs", "example_1.wav")) as w:
        assert w.getsampwidth() == 2 and w.getnchannels() == 1
        sr = w.getframerate()
        pcm = np.frombuffer(w.readframes(w.getnframes()), dtype="<i2").copy()
    audio = dict(conf["audio"])
    out = os.path.join(HERE, "scale_stats_ref.npz")
    np.savez(out, mel_mean=stats["mel_mean"], mel_std=stats["mel_std"], linear_mean=stats["linear_mean"],
             linear_std=stats["linear_std"], audio_config=json.dumps(stats["audio_config"]),
             test_audio=json.dumps(audio), wav_pcm16=pcm, wav_sr=np.int64(sr))
    print(out, {k: (v.shape, v.dtype) for k, v in stats.items() if isinstance(v, np.ndarray)},
          sorted(stats["audio_config"]))


if __name__ == "__main__":
    main()
