"""A batch of utterances over the GPUs of one node.

Utterances are independent: a batch is cut into per-GPU shards with no collective on the data
path. The shard plan is longest-processing-time first on a per-utterance cost (the decoder step
count, or the token count as its proxy before decoding: a shard's time is set by the longest
utterance in it, ``workload.lpt_shards``). Two ways to run the shards:

* ``GpuPool``: one worker process per GPU, spawned before the parent makes any GPU call, each
  holding its own models and library context; ``map`` sends every worker its shard and gathers the
  per-utterance results back into input order. ``Synthesizer`` uses it when its config asks for
  several GPUs (the per-sentence loop of ``TTS/server/synthesizer.py:144-183`` sharded).
* ``run_sharded``: inside a ``torch.distributed`` job with one process per GPU (``bench.py --gpus N``
  under torch.distributed.run): every rank derives the same plan, runs its shard, and the optional
  final gather brings every result to rank 0 (``gather_object``; over RCCL/xGMI with the nccl backend).
"""

import multiprocessing as mp
import os
import queue
import sys
import time
import traceback
from typing import Callable, List, Optional, Sequence

from .workload import lpt_shards


def shard_plan(costs: Sequence[float], n: int) -> List[List[int]]:
    """Index lists, one per GPU: LPT on ``costs`` with shard sizes differing by at most one."""
    if n < 1:
        raise ValueError("need at least one shard")
    return lpt_shards([float(c) for c in costs], n)


def run_sharded(runner: Callable[[list], list], items: Sequence, costs: Sequence[float], gather: bool = True,
                group=None):
    """Run this rank's LPT shard of ``items`` through ``runner`` (a list of items -> a list of
    results, one per item) and, with ``gather``, collect every rank's results on rank 0 in input
    order. Returns (results, mine): ``results`` is the full list on rank 0 (None elsewhere, or
    when gather is False), ``mine`` this rank's {index: result}."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    shard = shard_plan(costs, world)[rank]
    out = runner([items[i] for i in shard]) if shard else []
    if len(out) != len(shard):
        raise RuntimeError(f"runner returned {len(out)} results for {len(shard)} items")
    mine = dict(zip(shard, out))
    if not gather:
        return None, mine
    if world == 1:
        return [mine[i] for i in range(len(items))], mine
    parts = [None] * world if rank == 0 else None
    dist.gather_object(mine, parts, dst=0, group=group)
    if rank != 0:
        return None, mine
    merged = {}
    for p in parts:
        merged.update(p)
    return [merged[i] for i in range(len(items))], mine


def device_lock_path(device) -> str:
    """Lock file that serialises this library's runner calls on one GPU across processes
    (``TTS_GPU_LOCK_DIR``, default the temp directory)."""
    import tempfile
    d = os.environ.get("TTS_GPU_LOCK_DIR") or tempfile.gettempdir()
    return os.path.join(d, f"tts_amd_gpu{device}.lock")


class DeviceLock:
    """Inter-process exclusive lock on one device label (``fcntl.flock`` on ``device_lock_path``).

    The persistent decoder and BiLSTM launches hold every CU of their GPU for the whole call and
    meet at grid barriers: two such launches from different processes on one GPU can leave part of
    each grid waiting for CUs the other holds, and the barrier gives up after
    TTS_BARRIER_TIMEOUT_MS. Workers that share a device therefore run their calls
    one at a time under this lock."""

    def __init__(self, device):
        self.path = device_lock_path(device)
        self._fd = None

    def __enter__(self):
        import fcntl
        self._fd = os.open(self.path, os.O_RDWR | os.O_CREAT, 0o666)
        fcntl.flock(self._fd, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl
        fcntl.flock(self._fd, fcntl.LOCK_UN)
        os.close(self._fd)
        self._fd = None


def _pool_worker(factory, device, inq, outq):
    """Worker process: build the runner for ``device`` once, then serve shards until None. Every
    runner call holds the device's inter-process lock (``DeviceLock``)."""
    try:
        runner = factory(device)
        outq.put(("ready", device, None))
    except Exception:
        outq.put(("error", device, traceback.format_exc()))
        return
    while True:
        msg = inq.get()
        if msg is None:
            break
        job, idx, items, kw = msg
        try:
            with DeviceLock(device):
                res = runner(items, **kw)
            outq.put(("done", job, (idx, res)))
        except Exception:
            outq.put(("error", job, traceback.format_exc()))


class GpuPool:
    """One worker process per device. ``factory(device)`` (picklable: a module-level function or a
    functools.partial of one) builds the per-device runner inside the worker; the runner maps a list
    of items to a list of results. Create the pool before this process touches the GPU: workers are
    started with the 'spawn' method and initialise their own device (a GPU-initialised parent is
    refused). A device may be listed more than once: its workers' calls are serialised by a
    per-device inter-process lock (``DeviceLock``), so their grid-barrier launches never share the
    GPU at the same time."""

    POLL_S = 0.5  # how often map() checks that its workers are alive while it waits

    def __init__(self, factory: Callable, devices: Sequence[int], start_timeout: float = 600.0):
        if not devices:
            raise ValueError("GpuPool needs at least one device")
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            raise RuntimeError("GpuPool must be created before this process initialises the GPU "
                               "(spawned workers initialise their own device)")
        ctx = mp.get_context("spawn")
        self.devices = list(devices)
        self._out = ctx.Queue()
        self._in = [ctx.Queue() for _ in self.devices]
        self._procs = [ctx.Process(target=_pool_worker, args=(factory, d, q, self._out), daemon=True)
                       for d, q in zip(self.devices, self._in)]
        for p in self._procs:
            p.start()
        self._job = 0
        self._broken = None
        ready, errors = 0, []
        deadline = time.monotonic() + start_timeout
        while ready + len(errors) < len(self._procs):
            try:
                kind, dev, payload = self._out.get(timeout=self.POLL_S)
            except queue.Empty:
                dead = self._dead()
                if dead or time.monotonic() > deadline:
                    self.close()
                    raise RuntimeError("GpuPool worker failed to start: " +
                                       (f"worker for device(s) {dead} exited" if dead else "timed out"))
                continue
            if kind == "ready":
                ready += 1
            else:
                errors.append(f"device {dev}:\n{payload}")
        if errors:
            self.close()
            raise RuntimeError("GpuPool worker failed to start:\n" + "\n".join(errors))

    def _dead(self) -> List[int]:
        return [d for d, p in zip(self.devices, self._procs) if not p.is_alive()]

    def map(self, items: Sequence, costs: Optional[Sequence[float]] = None, timeout: float = 3600.0, **kw) -> list:
        """Results for ``items`` in input order; shards planned by LPT on ``costs`` (default: equal
        costs). Keyword arguments go to every runner call. A worker that dies, or a call past
        ``timeout`` seconds, raises and leaves the pool unusable (results of an abandoned call
        could still arrive)."""
        if self._broken:
            raise RuntimeError(f"GpuPool is unusable: {self._broken}")
        n = len(items)
        if n == 0:
            return []
        costs = [1.0] * n if costs is None else costs
        plan = shard_plan(costs, len(self.devices))
        self._job += 1
        job = self._job
        sent = 0
        for q, shard in zip(self._in, plan):
            if shard:
                q.put((job, shard, [items[i] for i in shard], kw))
                sent += 1
        out = [None] * n
        errors = []
        got = 0
        deadline = time.monotonic() + timeout
        while got < sent:
            try:
                kind, j, payload = self._out.get(timeout=self.POLL_S)
            except queue.Empty:
                dead = self._dead()
                if dead:
                    self._broken = f"worker for device(s) {dead} exited"
                    raise RuntimeError(f"GpuPool: {self._broken} during map()")
                if time.monotonic() > deadline:
                    self._broken = f"map() timed out after {timeout} s"
                    raise RuntimeError(f"GpuPool: {self._broken}")
                continue
            if j != job:  # a result of an earlier call that raised before it arrived
                continue
            got += 1
            if kind == "error":
                errors.append(payload)
                continue
            idx, res = payload
            if len(res) != len(idx):
                errors.append(f"runner returned {len(res)} results for {len(idx)} items")
                continue
            for i, r in zip(idx, res):
                out[i] = r
        if errors:
            raise RuntimeError("GpuPool worker failed:\n" + "\n".join(errors))
        return out

    def close(self):
        for q in self._in:
            try:
                q.put(None)
            except Exception:
                pass
        for p in self._procs:
            p.join(timeout=60)
            if p.is_alive():
                p.terminate()
        self._procs = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
