"""CPU, world sizes 2 and 4 over gloo: the multi-GPU bench path's partition and
timing logic (bench.py helpers) — barrier-bracketed timed region, max over
ranks, whole-job aggregate, and the round-robin frame deal."""
import os
import socket
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank 1 is the slow rank: 3 steps x 40 ms vs 3 x 5 ms
    delay = 0.040 if rank == 1 else 0.005
    el = bench.timed_region(lambda i: time.sleep(delay), 3, dist)
    mx = bench.max_over_ranks(el, dist)
    frames = list(bench.rank_frames(10, rank, world))
    q.put((rank, el, mx, frames))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_timing_and_partition():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, el0, mx0, f0), (r1, el1, mx1, f1) = res
    # both ranks agree on the max, and it is the slow rank's region
    assert mx0 == mx1 == max(el0, el1)
    assert mx0 >= 0.12
    # the barrier brackets the region: the fast rank waited for the slow one
    assert el0 >= 0.10
    # every frame dealt exactly once, round-robin
    assert sorted(f0 + f1) == list(range(10))
    assert f0 == [0, 2, 4, 6, 8] and f1 == [1, 3, 5, 7, 9]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_round_robin_deal_covers_every_frame(world):
    sys.path.insert(0, ROOT)
    import bench
    deals = [list(bench.rank_frames(37, r, world)) for r in range(world)]
    assert sorted(sum(deals, [])) == list(range(37))
    assert max(map(len, deals)) - min(map(len, deals)) <= 1


def test_aggregate_counts_all_ranks():
    sys.path.insert(0, ROOT)
    import bench
    v1 = bench.aggregate_gpix(1, 64, 4096, 4096, 20, 0.01)
    v8 = bench.aggregate_gpix(8, 64, 4096, 4096, 20, 0.01)
    assert v8 == pytest.approx(8 * v1)
    assert v1 == pytest.approx(64 * 4096 * 4096 * 20 / 0.01 / 1e9)


def _scatter_worker(rank, world, port, q):
    """Rank 0 owns all frames; scatter -> per-rank pyramid -> gather, on CPU
    tensors over gloo.  The per-rank compute here is the oracle (test
    infrastructure); on the GPU bench it is the HIP batch path."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    import oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B, H, W = 3, 24, 40
    fb = H * W * 4
    geo = [(40, 24, 1), (20, 12, 1), (10, 6, 1)]
    rng = np.random.default_rng(5)
    allf = rng.uniform(-1e3, 1e3, (world * B, H, W)).astype(np.float32)
    pool = torch.from_numpy(allf.view(np.uint8).reshape(-1).copy()) if rank == 0 else None
    local = torch.empty(B * fb, dtype=torch.uint8)
    mine = bench.scatter_frames(pool, local, fb, B, dist, rank, world)
    frames = mine.numpy().view(np.float32).reshape(B, H, W)
    lv = [None]
    for L in range(1, 3):
        w, h, _ = geo[L]
        outs = [oracle.cascade_2d(f, 3, 1)[L - 1] for f in frames]
        lv.append(torch.from_numpy(np.stack(outs).view(np.uint8).reshape(-1).copy()))
    pool_lv = [None] + [torch.empty(world * t.numel(), dtype=torch.uint8) for t in lv[1:]]
    bench.gather_levels(lv, pool_lv, dist, rank, world)
    if rank == 0:
        ok = True
        for L in range(1, 3):
            w, h, _ = geo[L]
            got = pool_lv[L].numpy().view(np.float32).reshape(world * B, h, w)
            for i in range(world * B):
                ok = ok and np.array_equal(got[i], oracle.cascade_2d(allf[i], 3, 1)[L - 1])
        q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_scatter_gather_logic(world):
    """Rank 0's pool scattered to `world` ranks and the levels gathered back
    in rank order (4 ranks rehearses the per-peer send loop beyond one peer)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok


@pytest.mark.parametrize("world", [2, 3, 4])
def test_resequence_round_robin(world):
    """Frames dealt round-robin come back in acquisition order: what the
    host must hand Array::write_frame (array.cpp:179-189)."""
    sys.path.insert(0, ROOT)
    import bench
    total = 23
    per_rank = [[("frame", i) for i in bench.rank_frames(total, r, world)] for r in range(world)]
    assert bench.resequence(per_rank, world) == [("frame", i) for i in range(total)]


def test_scatter_gather_are_grouped():
    """scatter_frames/gather_levels issue their point-to-point ops as one
    grouped batch (dist.batch_isend_irecv — RCCL group semantics, SURVEY
    §8(e)), never one isend/irecv at a time."""
    import inspect
    sys.path.insert(0, ROOT)
    import bench
    src = inspect.getsource(bench.grouped_p2p)
    assert "batch_isend_irecv" in src and "P2POp" in src
    for fn in (bench.scatter_frames, bench.gather_levels):
        src = inspect.getsource(fn)
        assert "grouped_p2p(" in src
        assert "dist.isend(" not in src and "dist.irecv(" not in src
