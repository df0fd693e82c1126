"""Benchmark workload and the multi-GPU shard plan (§8e).

* LJ profile: the 32 utterances of the reference's ``tests/data/ljspeech`` fixture, recorded
  in ``tests/golden/lj_profile.json`` (T_i = normalised-text length as a phoneme-count proxy,
  M_i = ceil(wav_samples / 256)).
* Token ids: ``numpy.random.RandomState(0).randint(1, 129, size=T_i)`` in file order.
* Forced length: stop bias -1e4 and ``max_decoder_steps_i = ceil(M_i / r)``.
* Sharding: utterances are independent units; a batch is split across ranks with no
  data-path collective. ``lpt_shards`` balances the per-shard max step count (batch time is
  set by the longest utterance in the shard).
"""

import json
import math
import os
from typing import List, Sequence

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROFILE = os.path.join(_ROOT, "tests", "golden", "lj_profile.json")
SAMPLE_RATE = 22050
HOP = 256


def lj_profile(path: str = PROFILE):
    with open(path) as f:
        rows = json.load(f)["utterances"]
    return [r["T"] for r in rows], [r["M"] for r in rows]


def synthetic_ids(T_list: Sequence[int], seed: int = 0, num_chars: int = 129) -> List[np.ndarray]:
    rs = np.random.RandomState(seed)
    return [rs.randint(1, num_chars, size=T).astype(np.int64) for T in T_list]


def forced_steps(M_list: Sequence[int], r: int) -> List[int]:
    return [int(math.ceil(M / r)) for M in M_list]


def pad_batch(ids: Sequence[np.ndarray]):
    T = max(len(x) for x in ids)
    out = np.zeros((len(ids), T), np.int64)
    for i, x in enumerate(ids):
        out[i, :len(x)] = x
    return out, np.array([len(x) for x in ids], np.int64)


def lpt_shards(costs: Sequence[float], n: int) -> List[List[int]]:
    """Longest-processing-time-first assignment of items to n shards of equal count.

    Each shard gets ceil(len/n) or floor(len/n) items; items are taken longest first and
    placed on the open shard with the smallest current load. Returns sorted index lists.
    """
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    cap = [len(costs) // n + (1 if k < len(costs) % n else 0) for k in range(n)]
    load = [0.0] * n
    shards: List[List[int]] = [[] for _ in range(n)]
    for i in order:
        k = min((k for k in range(n) if len(shards[k]) < cap[k]), key=lambda k: (load[k], k))
        shards[k].append(i)
        load[k] += costs[i]
    return [sorted(s) for s in shards]


def replicated_workload(world_size: int, per_rank: int = 32):
    """C3: the 32-utterance profile replicated world_size times (per-rank batch 32).

    Every rank gets exactly one copy, i.e. the LPT split of identical copies; returns the
    global (T, M) lists and each rank's index list.
    """
    T, M = lj_profile()
    assert per_rank % len(T) == 0 or len(T) % per_rank == 0
    reps = max(1, (per_rank * world_size) // len(T))
    T_all = T * reps
    M_all = M * reps
    shards = [list(range(k * per_rank, (k + 1) * per_rank)) for k in range(world_size)]
    return T_all, M_all, shards
