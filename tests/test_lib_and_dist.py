"""CPU: the C-ABI library loads and exports every symbol include/ttship.h declares (no compute
calls without a GPU), and the N>1 path (utterance sharding + final gather) on a world_size-2
gloo group running the oracle."""
import os
import re
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "ttship.h")).read()
    return sorted(set(re.findall(r"\b(tts_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from tts_amd._lib import SIGNATURES, load_library
    lib = load_library()
    declared = _declared_symbols()
    assert len(declared) >= 14
    for name in declared:
        assert hasattr(lib, name), f"libttship.so does not export {name}"
    assert sorted(n for n, _, _ in SIGNATURES) == declared
    assert lib.tts_version() == 1
    assert isinstance(lib.tts_last_error(), bytes)


def test_library_is_gfx950_code_object():
    path = os.path.join(ROOT, "tts_amd", "libttship.so")
    blob = open(path, "rb").read()
    assert b"gfx950" in blob


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


STEPS = [5, 2, 4, 3, 2, 4]


def test_lpt_shards_balance_steps():
    from tts_amd.workload import lpt_shards
    sh = lpt_shards([float(s) for s in STEPS], 2)
    assert sorted(sum(sh, [])) == list(range(len(STEPS))) and all(len(x) == 3 for x in sh)
    loads = [sum(STEPS[i] for i in x) for x in sh]
    assert max(loads) - min(loads) <= max(STEPS) - min(STEPS)
    assert {max(STEPS[i] for i in x) for x in sh} == {5, 4}  # the two longest land on different ranks


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from helpers import taco_state_dict
    from oracle.taco_np import TacoOracle
    from tts_amd.spec import TacotronConfig
    from tts_amd.workload import lj_profile, lpt_shards, synthetic_ids
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=2, overrides={}, stop_bias=-1e4, cfg=cfg)
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    T, _ = lj_profile()
    T = [min(t, 12) for t in T[:6]]             # 6 short utterances with their own step counts
    ids = synthetic_ids(T)
    # shards balance the decoder step counts (a batch's time is set by its decode length)
    # the product entry point (tts_amd.multigpu.run_sharded): this rank's LPT shard through the
    # runner, no collective on the data path, then the optional final gather to rank 0
    from tts_amd.multigpu import run_sharded, shard_plan
    assert shard_plan([float(s) for s in STEPS], world) == lpt_shards([float(s) for s in STEPS], world)
    items = list(zip(ids, STEPS))
    res, mine = run_sharded(lambda xs: [orc.inference(x, 2, s)[1] for x, s in xs], items, STEPS)
    assert sorted(mine) == lpt_shards([float(s) for s in STEPS], world)[rank]
    if rank == 0:
        M = 2 * max(STEPS)
        buf = np.zeros((len(T), M, 80), np.float32)
        for i, p in enumerate(res):
            buf[i, :len(p)] = p
        q.put(buf)
    else:
        assert res is None
    dist.destroy_process_group()


def test_two_rank_sharded_decode_equals_single_process():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from helpers import taco_state_dict
    from oracle.taco_np import TacoOracle
    from tts_amd.spec import TacotronConfig
    from tts_amd.workload import lj_profile, synthetic_ids
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=2, overrides={}, stop_bias=-1e4, cfg=cfg)
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)
    T, _ = lj_profile()
    ids = synthetic_ids([min(t, 12) for t in T[:6]])
    for i in range(6):
        ref = orc.inference(ids[i], 2, STEPS[i])[1]
        assert np.array_equal(out[i, :len(ref)], ref) and not out[i, len(ref):].any()


def _bench_rank_worker(rank, world, port, q):
    """One rank of bench.py's multi-GPU path on gloo: its shard selection (rank_shard), a stub step
    loop timed as bench.py times it (barrier, per-rank elapsed time, MAX / SUM aggregation) and the
    line's config."""
    import sys
    import time
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from tts_amd.workload import forced_steps
    r, n = 2, 3
    mine, my_T, my_prof, M_all = bench.rank_shard(world, rank, 32, r)
    steps = forced_steps([M_all[i] for i in mine], r)
    dist.barrier()
    t0 = time.perf_counter()
    frames = 0
    for _ in range(n):  # stub step: the rank's mel frames, and a rank-dependent duration
        time.sleep(0.02 * (rank + 1))
        frames += sum(st * r for st in steps)
    dist.barrier()
    el = time.perf_counter() - t0
    ms, per = bench.aggregate(el, frames, n, world, torch.device("cpu"))
    q.put((rank, mine, my_prof, my_T, steps, el, ms, per, bench.bench_config(world, 32, r)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bench_multi_rank_shards_and_aggregation(world):
    """bench.py at N > 1 (the driver's 8-GPU SCALE run): every rank holds one copy of every profile
    utterance, the ranks' shards partition the global batch, the line's time is the slowest rank's
    and its frame count the sum over ranks, and config.global_batch = 32 N."""
    from tts_amd.workload import forced_steps, lj_profile
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_rank_worker, args=(k, world, port, q)) for k in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    T, M = lj_profile()
    all_idx = sorted(i for _, mine, *_ in res for i in mine)
    assert all_idx == list(range(32 * world))  # a partition of the global batch
    per_rank_frames = sum(forced_steps(M, 2)) * 2
    max_el = max(el for *_, el, _, _, _ in res)
    for rank, mine, prof, my_T, steps, el, ms, per, cfg in res:
        assert sorted(prof) == list(range(32)), f"rank {rank} does not hold one copy of each utterance"
        assert sorted(my_T) == sorted(T) and sum(steps) * 2 == per_rank_frames
        assert per == world * per_rank_frames
        assert ms == pytest.approx(max_el / 3 * 1000.0, rel=1e-9)
        assert cfg["global_batch"] == 32 * world and cfg["parallelism"] == f"replicas x{world}"
        assert cfg["workload"].startswith("C3")


def test_bench_launch_decision():
    """`python bench.py --gpus N` (the driver's command form): with no WORLD_SIZE and N > 1 it
    becomes the launcher of N ranks (torch.distributed.run as a child, same arguments); inside a
    launcher's rank it runs itself; a WORLD_SIZE that differs from --gpus is refused."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    argv = ["--gpus", "2", "--steps", "3", "--no-cpu-baseline"]
    cmd = bench.launch_plan(2, {}, argv)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv) - 1] == os.path.join(ROOT, "bench.py") and cmd[-len(argv):] == argv
    assert bench.launch_plan(2, {"MASTER_PORT": "29511"}, argv)[cmd.index("--master-port") + 1] == "29511"
    assert bench.launch_plan(1, {}, ["--gpus", "1"]) is None
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}, argv) is None
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, argv) is None
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        bench.launch_plan(2, {"WORLD_SIZE": "4"}, argv)
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {}, argv)


def test_bench_gpus_2_starts_two_ranks_plan_only():
    """End to end on the CPU: `python bench.py --gpus 2 --plan-only` from a process with no
    WORLD_SIZE starts two ranks under torch.distributed.run; each prints its own shard of the
    64-utterance C3 batch before touching a GPU, and the shards partition it."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--plan-only"],
                         env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1] and all(d["world"] == 2 for d in lines)
    assert sorted(i for d in lines for i in d["shard"]) == list(range(64))
    # a mismatched launcher is refused with a nonzero status
    env["WORLD_SIZE"] = "3"
    bad = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--plan-only"],
                         env=env, capture_output=True, text=True, timeout=600)
    assert bad.returncode != 0 and "WORLD_SIZE=3" in bad.stderr


def _pool_factory(seed, device):
    """GpuPool stand-in runner for the CPU suite: the oracle decode, tagged with the worker's device."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import taco_state_dict
    from oracle.taco_np import TacoOracle
    from tts_amd.spec import TacotronConfig
    cfg = TacotronConfig()
    _, sd = taco_state_dict(None, seed=seed, overrides={}, stop_bias=-1e4, cfg=cfg)
    orc = TacoOracle(sd, cfg.attn_norm, cfg.r)

    def run(items, r=2):
        return [(device, orc.inference(x, r, s)[1]) for x, s in items]
    return run


def test_gpu_pool_dispatch_and_gather():
    """tts_amd.multigpu.GpuPool: one spawned worker per device label, LPT shards on the step counts,
    results gathered back in input order and equal to one process; a failing worker raises."""
    import functools
    from tts_amd.multigpu import GpuPool, shard_plan
    from tts_amd.workload import lj_profile, synthetic_ids
    T, _ = lj_profile()
    ids = synthetic_ids([min(t, 12) for t in T[:6]])
    items = list(zip(ids, STEPS))
    with GpuPool(functools.partial(_pool_factory, 2), devices=[0, 1]) as pool:
        out = pool.map(items, costs=STEPS)
        plan = shard_plan(STEPS, 2)
        for k, shard in enumerate(plan):
            assert all(out[i][0] == k for i in shard)
        ref = _pool_factory(2, -1)(items)
        for (_, a), (_, b) in zip(out, ref):
            assert np.array_equal(a, b)
        assert pool.map([]) == []
        with pytest.raises(RuntimeError, match="worker failed"):
            pool.map(items, r=0)  # r = 0 raises inside the workers


def _interval_factory(device):
    """GpuPool stand-in runner that records when each call ran (for the device-lock test)."""
    import time

    def run(items, hold=0.4):
        t0 = time.monotonic()
        if any(x == "die" for x in items):
            os._exit(3)  # a worker that dies mid-call (GPU fault stand-in)
        time.sleep(hold)
        return [(device, os.getpid(), t0, time.monotonic()) for _ in items]
    return run


def test_gpu_pool_serialises_workers_sharing_a_device(tmp_path, monkeypatch):
    """Two workers on one device label: their runner calls never overlap (per-device inter-process
    lock, tts_amd.multigpu.DeviceLock); workers on different labels run concurrently."""
    from tts_amd.multigpu import GpuPool
    monkeypatch.setenv("TTS_GPU_LOCK_DIR", str(tmp_path))
    with GpuPool(_interval_factory, devices=[0, 0]) as pool:
        for _ in range(2):
            out = pool.map(["a", "b"])
            (d0, p0, s0, e0), (d1, p1, s1, e1) = out
            assert d0 == d1 == 0 and p0 != p1
            assert e0 <= s1 or e1 <= s0, f"calls on one device overlapped: {out}"
    with GpuPool(_interval_factory, devices=[0, 1]) as pool:
        out = pool.map(["a", "b"], hold=1.5)
        (d0, _, s0, e0), (d1, _, s1, e1) = out
        assert {d0, d1} == {0, 1}
        assert s1 < e0 and s0 < e1, "workers on different devices were serialised"


def test_gpu_pool_dead_worker_and_gpu_parent(monkeypatch, tmp_path):
    """A worker that dies during map() raises a RuntimeError naming its device and leaves the pool
    unusable; a parent that has initialised the GPU is refused."""
    import torch
    from tts_amd.multigpu import GpuPool
    monkeypatch.setenv("TTS_GPU_LOCK_DIR", str(tmp_path))
    pool = GpuPool(_interval_factory, devices=[0, 1])
    try:
        with pytest.raises(RuntimeError, match=r"device\(s\) \[\d\] exited"):
            pool.map(["ok", "die"], hold=0.1)
        with pytest.raises(RuntimeError, match="unusable"):
            pool.map(["ok"])
    finally:
        pool.close()
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    with pytest.raises(RuntimeError, match="before this process initialises the GPU"):
        GpuPool(_interval_factory, devices=[0])


def test_library_matches_build_record():
    """__graft_entry__.build() records which sources libttship.so was built from; the library that
    loads must be that build of this tree's sources (no stale .so)."""
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    if not os.path.exists(g.BUILD_INFO):
        pytest.skip("library not built through __graft_entry__.build()")
    assert "built" in g.build_check()
