"""bench.py — device-resident multiscale downsample throughput on MI355X.

Metric (BASELINE.json): GPixels/s device-resident multiscale downsample,
4096^2 uint16, 5 levels.  GPix/s counts base-level pixels
(frames x W x H / time).  One "step" = one pass of the hot path over one
batch of B frames already resident in HBM on every rank: the whole pyramid
(levels 1..4) of every frame, written to HBM.  It is one fused cascade
launch per step (aqz_ds_run_device_batch).

Multi-GPU: one process per GPU (torchrun); frames are independent, so each
rank runs its own batch with no data-path collective (weak scaling); the
barrier and the max-over-ranks of the timed region use torch.distributed.

Rank 0 prints ONE JSON line.  Besides the contract fields it carries
`roofline` (algorithmic bytes / average kernel duration from HIP events on the
launch stream, against the 8 TB/s HBM peak), `cpu_baseline` (the reference's
own downsampler.cpp, compiled unmodified into oracle/_ref, on one core over a
bounded sample on this host, with the oracle port timed beside it), and `e2e` (host frame -> pinned H2D -> kernels -> D2H -> take_frame
through the streaming API, the path's real end-to-end rate).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

WORKLOADS = {
    # name: (width, height, planes, dtype, xy chunk, z chunk, frames per step)
    # planes = 0: 2-D frames; levels always come from the planner.
    "4096x4096_u16": (4096, 4096, 0, np.uint16, 256, 0, 64),     # headline, configs[2]
    "2048x2048_u16": (2048, 2048, 0, np.uint16, 256, 0, 64),     # configs[1]
    # configs[3] (per GPU): 128 frames (8 GiB in) run 2-3% faster per frame
    # than 64 for every method, where the u16 headline is fastest at 64
    # (profiles/r05/fbatch/)
    "4096x4096_f32": (4096, 4096, 0, np.float32, 256, 0, 128),
    "512x512_u8": (512, 512, 0, np.uint8, 128, 0, 1024),         # configs[0] synthetic
    # configs[4]: four 256-plane volumes (timepoints) per step.  In HBM,
    # Decimate over four takes 37 us per volume against 43 for one (the unit
    # order of DESIGN.md §11.11); Mean/Min/Max run alike either way.
    "1024x1024x256_u16": (1024, 1024, 256, np.uint16, 256, 64, 1024),
    # not BASELINE configs: the other element widths at the headline size
    "4096x4096_u32": (4096, 4096, 0, np.uint32, 256, 0, 64),
    "4096x4096_f64": (4096, 4096, 0, np.float64, 256, 0, 32),
}
HEADLINE_METRIC = "GPixels/s device-resident multiscale downsample, 4096² uint16, 5 levels"


# ---- distributed helpers (covered on CPU by tests/test_distributed.py) ----

def rank_frames(total_frames: int, rank: int, world: int):
    """Round-robin deal of one acquisition stream over ranks: frame i goes to
    rank i % world (frames are independent)."""
    return range(rank, total_frames, world)


def timed_region(step, steps: int, dist=None, sync=lambda: None):
    """Barrier + device sync on both sides of exactly `steps` calls of
    step(i); returns this rank's wall time in seconds."""
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    sync()
    if dist is not None:
        dist.barrier()
    return time.perf_counter() - t0


def max_over_ranks(value: float, dist=None, device="cpu") -> float:
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_gpix(world: int, frames_per_rank: int, W: int, H: int, steps: int,
                   elapsed_max: float) -> float:
    """Whole-job base GPixels/s: every rank's frames over the slowest rank."""
    return world * frames_per_rank * W * H * steps / elapsed_max / 1e9


def grouped_p2p(dist, ops):
    """One grouped point-to-point batch: `ops` = [("send"|"recv", tensor,
    peer)].  Under nccl (RCCL) it is dist.batch_isend_irecv — ncclGroupStart,
    every send/recv, ncclGroupEnd — so all peers' xGMI links stream at once.
    gloo moves host memory only: device tensors are staged through host
    copies there (the one-GPU rehearsal of the N-rank path)."""
    if not ops:
        return
    staged = []
    p2p = []
    host = dist.get_backend() != "nccl"
    for kind, t, peer in ops:
        if host and t.is_cuda:
            h = t.cpu() if kind == "send" else t.new_empty(t.shape, device="cpu")
            if kind == "recv":
                staged.append((t, h))
            t = h
        p2p.append(dist.P2POp(dist.isend if kind == "send" else dist.irecv, t, peer))
    for q in dist.batch_isend_irecv(p2p):
        q.wait()
    for dev, h in staged:
        dev.copy_(h)


def scatter_frames(pool, local, frame_bytes: int, frames_per_rank: int, dist,
                   rank: int, world: int):
    """Batched-frame config F over xGMI: rank 0 holds every
    rank's frames contiguously in `pool` (rank r's block at r*frames_per_rank)
    and sends each block to its rank as ONE grouped point-to-point batch
    (grouped_p2p).  Returns the tensor this rank computes on."""
    blk = frames_per_rank * frame_bytes
    if rank == 0:
        grouped_p2p(dist, [("send", pool[r * blk:(r + 1) * blk], r) for r in range(1, world)])
        return pool[:blk]
    grouped_p2p(dist, [("recv", local[:blk], 0)])
    return local[:blk]


def gather_levels(level_bufs, pool_levels, dist, rank: int, world: int):
    """Every rank's level outputs back to rank 0 in one grouped p2p batch
    (all levels, all peers); rank 0 lays rank r's block of level L at
    pool_levels[L][r*len:(r+1)*len] (its own block is copied locally).
    Blocks are contiguous frame ranges in rank order, so rank 0's levels come
    back in acquisition order — the order Array::write_frame requires
    (array.cpp:179-189 rejects out-of-order frame ids)."""
    ops = []
    for L, buf in enumerate(level_bufs):
        if buf is None:
            continue
        n = buf.numel()
        if rank == 0:
            pool_levels[L][:n].copy_(buf)
            ops += [("recv", pool_levels[L][r * n:(r + 1) * n], r) for r in range(1, world)]
        else:
            ops.append(("send", buf, 0))
    grouped_p2p(dist, ops)


def resequence(per_rank_frames, world: int):
    """Acquisition order from a round-robin deal (rank_frames): frame i came
    back as the (i // world)-th frame of rank i % world.  The host side of
    frame sharding without a gather: levels reach the writer
    in frame-id order, as Array::write_frame requires (array.cpp:179-189)."""
    total = sum(len(f) for f in per_rank_frames)
    return [per_rank_frames[i % world][i // world] for i in range(total)]


def algorithmic_bytes(geo, counts, frames: int, method: str, bpp: int, tile=None):
    """(read, read + written) algorithmic bytes of one batch step (SURVEY
    §8(d)): every input frame read once, every emitted level frame
    (counts[L] of level L) written once — with `tile` = (rows, cols), as
    whole chunk tiles, zero overhang included.  Decimate keeps the top-left
    pixel and the earlier plane, so only the even rows (and, where level 1
    halves Z, the even planes) are needed; whole rows, because the sampled
    columns share 64-B bursts with the skipped ones.  Every other method
    reads all."""
    W, H, planes0 = geo[0]
    read = frames * W * H * bpp
    if method == "decimate" and len(geo) > 1:
        rows = (H + 1) // 2 if geo[1][0] < W or geo[1][1] < H else H
        planes = (frames + 1) // 2 if geo[1][2] < planes0 else frames
        read = planes * rows * W * bpp
    if tile:
        tr, tc = tile
        written = sum(counts[L] * (-(-geo[L][0] // tc)) * (-(-geo[L][1] // tr)) * tr * tc * bpp
                      for L in range(1, len(geo)))
    else:
        written = sum(counts[L] * geo[L][0] * geo[L][1] * bpp for L in range(1, len(geo)))
    return read, read + written


class stdout_to_stderr:
    """Send file descriptor 1 to stderr inside the block: gloo's C++ code
    prints its connection messages ("[Gloo] Rank 0 is connected to ...") on
    stdout, which must carry rank 0's JSON line alone."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(argv, gpus: int, port: int):
    """`python -m torch.distributed.run` starting `gpus` ranks of this script
    with the same arguments (one process per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1",
            f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def resolve_world(args, env):
    """('launch', N) when this process must start N ranks itself, ('run', N)
    when it is one of N ranks (or the only one); raises SystemExit when
    --gpus contradicts the launcher's WORLD_SIZE."""
    world = env.get("WORLD_SIZE")
    if world is None:
        n = args.gpus or 1
        return ("launch", n) if n > 1 else ("run", 1)
    world = int(world)
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started "
                         f"WORLD_SIZE={world} ranks")
    return ("run", world)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (ranks) of one node; N > 1 without a launcher "
                        "starts N ranks via torch.distributed.run (default: "
                        "WORLD_SIZE, else 1)")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", default="4096x4096_u16", choices=sorted(WORKLOADS))
    p.add_argument("--batch", type=int, default=0,
                   help="frames (planes) per step per GPU; 0 = workload default")
    p.add_argument("--method", default="mean", choices=["decimate", "mean", "min", "max"])
    p.add_argument("--rotate-mib", type=int, default=1024,
                   help="launches cycle over copies of the input and output buffers "
                        "until the bytes a launch reads, over all copies, reach this "
                        "many MiB (4x the 256 MB Infinity Cache by default), so that "
                        "no launch finds its input left in the cache by the launch "
                        "before; 0: one buffer set")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="bounded CPU-baseline sample (0 disables)")
    p.add_argument("--e2e-frames", type=int, default=48,
                   help="frames through the streaming host API (0 disables)")
    p.add_argument("--no-check", action="store_true",
                   help="skip the one-frame oracle spot check")
    p.add_argument("--no-pmc", action="store_true",
                   help="skip the rocprofv3 FETCH_SIZE/WRITE_SIZE traffic passes")
    p.add_argument("--sink", default="",
                   help="directory for the filesystem-sink legs (default: a temporary "
                        "directory): BASELINE config C2 (2048^2 u16, 4 levels) always, "
                        "and with --sink also the workload itself; raw level files, "
                        "fsync'd")
    p.add_argument("--xgmi-scatter", action="store_true",
                   help="BASELINE config F through the library: every step, rank 0's "
                        "batch of (GPUs x B) frames is sharded over the node's GPUs by "
                        "aqz_node_run_device_batch (peer copies over xGMI, levels back "
                        "in frame order); rank 0 drives every GPU, the other ranks "
                        "wait; timed end to end")
    p.add_argument("--node-devices", default="",
                   help="--xgmi-scatter: HIP ordinals of the node's handles (default: "
                        "one per rank); repeat one to rehearse on a smaller box, "
                        "e.g. 0,0")
    p.add_argument("--stage-all", action="store_true",
                   help="--xgmi-scatter: every block takes the remote-GPU staging path, "
                        "also on the batch's own GPU (AQZ_NODE_STAGE_ALL)")
    p.add_argument("--xgmi-rccl", action="store_true",
                   help="N>1 only: the same scatter/gather as torch.distributed RCCL "
                        "p2p between the rank processes instead (one rank per GPU)")
    p.add_argument("--tiled", action="store_true",
                   help="emit every level chunk-tiled (chunk x chunk tiles) from the "
                        "pyramid kernel itself: aqz_ds_run_device_batch_tiled "
                        "(SURVEY §8(f) row 2); 2-D workloads")
    p.add_argument("--chunk", type=int, default=0,
                   help="override the workload's XY chunk size (level planning and --tiled tiles)")
    p.add_argument("--no-flags", action="store_true",
                   help="--tiled without the chunk zero scan (A/B of its cost)")
    p.add_argument("--shape", default="",
                   help="WxH: override the workload's frame size (same dtype, chunk "
                        "and batch bytes), e.g. 5472x3648")
    p.add_argument("--per-launch-events", action="store_true",
                   help="an event pair around every launch (per-launch min; adds a "
                        "~12 us gap between kernels)")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args(argv)


def main():
    args = parse()
    mode, world = resolve_world(args, os.environ)
    if mode == "launch":
        # Before torch, the library or any GPU call: the ranks run as a child
        # process (never exec from a process that may touch the GPU); rank 0's
        # JSON line reaches stdout through the inherited descriptors.
        import subprocess
        rc = subprocess.run(launcher_cmd(sys.argv[1:], world, free_port())).returncode
        sys.exit(rc)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch  # plumbing: device buffers, events, process group
    import aqz_pkg
    aqz = aqz_pkg.load()
    aqz.lib()  # fail loudly if the native library is missing

    # one GPU per rank; the modulo only matters when rehearsing N>1 on a
    # smaller box (AQZ_DIST_BACKEND=gloo, ranks sharing a device)
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("AQZ_DIST_BACKEND", "nccl")  # nccl = RCCL
        with stdout_to_stderr():
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", device))
            else:
                dist.init_process_group(backend)

    W, H, Z, dtype, chunk, zchunk, default_batch = WORKLOADS[args.workload]
    if args.shape:
        # same batch bytes as the workload's default batch
        W2, H2 = (int(x) for x in args.shape.lower().split("x"))
        default_batch = max(1, default_batch * W * H // (W2 * H2))
        W, H = W2, H2
    if args.chunk:
        chunk = args.chunk
    if args.tiled and Z:
        raise SystemExit("--tiled: 2-D workloads only")
    method = aqz.METHODS[args.method]
    dims = [(aqz.TIME, 0, 1, 1)]
    if Z:
        dims.append((aqz.SPACE, Z, zchunk, 1))
    dims += [(aqz.SPACE, H, chunk, 1), (aqz.SPACE, W, chunk, 1)]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    n_levels = len(geo)
    bpp = np.dtype(dtype).itemsize
    B = args.batch or default_batch
    frame_bytes = W * H * bpp
    n_rot = rotation_copies(B * frame_bytes, args.method, bool(Z), args.rotate_mib)
    if args.xgmi_scatter or args.xgmi_rccl:
        n_rot = 1  # these modes keep one buffer set (their batches are >= 2 GiB)

    # synthetic input, resident in HBM before timing (seeded per rank);
    # n_rot copies of it at distinct addresses (copy 0 is `d_in`)
    gen = torch.Generator(device="cuda").manual_seed(0xA0C2A11 + rank)
    d_all = torch.empty(n_rot * B * frame_bytes, dtype=torch.uint8, device="cuda")
    d_in = d_all[:B * frame_bytes]
    if np.dtype(dtype).kind == "f":
        tdt = torch.float64 if np.dtype(dtype).itemsize == 8 else torch.float32
        d_in.view(tdt).copy_(torch.rand(B * W * H, device="cuda", generator=gen, dtype=tdt)
                             * 2000 - 1000)
    else:
        d_in.copy_(torch.randint(0, 256, (B * frame_bytes,), dtype=torch.uint8,
                                 device="cuda", generator=gen))
    for k in range(1, n_rot):
        d_all[k * B * frame_bytes:(k + 1) * B * frame_bytes].copy_(d_in)
    ds = aqz.Downsampler(geo, dtype, method, device=device)
    if args.tiled:
        # chunk x chunk tiles per level, zero overhang included
        tile_elems = [0] + [(-(-w // chunk)) * (-(-h // chunk)) * chunk * chunk
                            for w, h, _ in geo[1:]]
        outs = [None] + [torch.empty(B * e * bpp, dtype=torch.uint8, device="cuda")
                         for e in tile_elems[1:]]
        flag_slots = [0] + [ds.tiled_flag_slots(L, chunk, chunk) for L in range(1, n_levels)]
        flags = [None] + [torch.empty(B * e // (chunk * chunk) * flag_slots[L],
                                      dtype=torch.uint8, device="cuda")
                          for L, e in enumerate(tile_elems[1:], 1)]
        flag_ptrs = None if args.no_flags else [0] + [f.data_ptr() for f in flags[1:]]
    else:
        outs = [None] + [torch.empty(B * w * h * bpp, dtype=torch.uint8, device="cuda")
                         for w, h, _ in geo[1:]]
    out_ptrs = [0] + [o.data_ptr() for o in outs[1:]]
    # output sets of the other copies (set 0 is `outs`, the checked one)
    rot_outs = [[None] + [torch.empty_like(o) for o in outs[1:]] for _ in range(1, n_rot)]
    rot_flags = ([[None] + [torch.empty_like(f) for f in flags[1:]] for _ in range(1, n_rot)]
                 if args.tiled and flag_ptrs is not None else None)
    # A real (non-null) stream: the kernels run on it and the timing events
    # are recorded on it.
    torch.cuda.synchronize()  # inputs were generated on the default stream
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    assert sptr, "need a non-null HIP stream"

    counts = [0] * n_levels
    xgmi = args.xgmi_rccl and dist is not None
    # --xgmi-scatter: the library's node over the node's GPUs, from rank 0
    node_devices = None
    if args.xgmi_scatter:
        node_devices = ([int(x) for x in args.node_devices.split(",")] if args.node_devices
                        else list(range(world)))
        if len(node_devices) < 2:
            raise SystemExit("--xgmi-scatter: needs two or more GPUs (ranks or --node-devices)")
    xnode = None
    if node_devices is not None and rank == 0:
        ND = len(node_devices)
        pool = torch.empty(ND * B * frame_bytes, dtype=torch.uint8, device="cuda")
        for r in range(ND):
            pool[r * B * frame_bytes:(r + 1) * B * frame_bytes].copy_(d_in)
        pool_levels = [None] + [torch.empty(ND * o.numel(), dtype=torch.uint8, device="cuda")
                                for o in outs[1:]]
        torch.cuda.synchronize()
        node = aqz.Node(geo, dtype, method, node_devices)
        xnode = {"node": node, "pool": pool, "levels": pool_levels, "n": ND,
                 "call": node.device_batch_call(pool.data_ptr(), device, ND * B,
                                                [0] + [t.data_ptr() for t in pool_levels[1:]],
                                                sptr, stage_all=args.stage_all),
                 "counts": None}
    if xgmi:
        # config F: rank 0's pool holds every rank's frames; levels return
        # to rank 0.  Rank 0 computes on the first block of its pool.
        if rank == 0:
            pool = torch.empty(world * B * frame_bytes, dtype=torch.uint8, device="cuda")
            for r in range(world):
                pool[r * B * frame_bytes:(r + 1) * B * frame_bytes].copy_(d_in)
            pool_levels = [None] + [torch.empty(world * o.numel(), dtype=torch.uint8,
                                                device="cuda") for o in outs[1:]]
        else:
            pool, pool_levels = None, None

    # one prepared foreign call per step: short launches (small frames) would
    # otherwise wait on Python building ctypes arrays between them
    if args.tiled:
        batch = ds.batch_call(d_in.data_ptr(), B, out_ptrs, sptr,
                              tiles=[None] + [(chunk, chunk)] * (n_levels - 1),
                              device_nonzero=flag_ptrs)
    else:
        batch = ds.batch_call(d_in.data_ptr(), B, out_ptrs, sptr)
    # one call per buffer copy; steps take them in turn (copy 0 first)
    def copy_call(k):
        src = d_all.data_ptr() + k * B * frame_bytes
        ptrs = [0] + [o.data_ptr() for o in rot_outs[k - 1][1:]]
        if not args.tiled:
            return ds.batch_call(src, B, ptrs, sptr)
        return ds.batch_call(src, B, ptrs, sptr,
                             tiles=[None] + [(chunk, chunk)] * (n_levels - 1),
                             device_nonzero=(None if rot_flags is None else
                                             [0] + [f.data_ptr() for f in rot_flags[k - 1][1:]]))
    batches = [batch] + [copy_call(k) for k in range(1, n_rot)]
    turn = [0]

    def step(ev=None):
        """One step; `ev` = (start, kernel_start, kernel_end, end) events
        recorded on the launch stream, so that in --xgmi-rccl mode the
        kernel's own time is separate from the p2p scatter/gather around it
        (the p2p work is joined onto `stream` by wait())."""
        if node_devices is not None:
            # the whole node's batch from rank 0 (the other ranks idle)
            if xnode is not None:
                if ev:
                    ev[1].record(stream)
                xnode["counts"] = xnode["call"]()
                if ev:
                    ev[2].record(stream)
        elif xgmi:
            if ev:
                ev[0].record(stream)
            mine = scatter_frames(pool, d_in, frame_bytes, B, dist, rank, world)
            if ev:
                ev[1].record(stream)
            counts[:] = ds.run_device_batch(mine.data_ptr(), B, out_ptrs, sptr)
            if ev:
                ev[2].record(stream)
            gather_levels(outs, pool_levels, dist, rank, world)
            if ev:
                ev[3].record(stream)
        else:
            if ev:
                ev[1].record(stream)
            counts[:] = batches[turn[0] % n_rot]()
            turn[0] += 1
            if ev:
                ev[2].record(stream)

    if args.pmc_child:
        # launched under `rocprofv3 --pmc` by measure_traffic(): launches only
        for _ in range(args.warmup + args.steps):
            step()
        torch.cuda.synchronize()
        ds.close()
        return

    # correctness spot check of one frame against the oracle (rank 0, N=1)
    check = None
    if not args.no_check:
        turn[0] = 0  # the checked outputs are copy 0's
        step()  # every rank: in --xgmi-scatter mode the step is collective
        torch.cuda.synchronize()
    if not args.no_check and rank == 0:
        import oracle as orc_mod  # test infrastructure: checker only
        # first 2^(levels-1) frames (one aligned plane group for volumes)
        nchk = min(B, 1 << (n_levels - 1)) if Z else 1
        host = d_in[:nchk * frame_bytes].cpu().numpy().view(dtype).reshape(nchk, H, W)
        ref = orc_mod.OracleDownsampler(geo, dtype, method)
        emitted = [0] * n_levels
        ok = True
        for i in range(nchk):
            ref.add_frame(host[i])
            for L in range(1, n_levels):
                r = ref.take_frame(L)
                if r is None:
                    continue
                w, h, _ = geo[L]
                k = emitted[L]
                if args.tiled:
                    e = tile_elems[L] * bpp
                    got = outs[L][k * e:(k + 1) * e].cpu().numpy()
                    t, nz = orc_mod.tile_frame(r, chunk, chunk)
                    S = flag_slots[L]
                    ok = ok and np.array_equal(got, t.view(np.uint8).reshape(-1))
                    if not args.no_flags:
                        gf = flags[L][k * len(nz) * S:(k + 1) * len(nz) * S].cpu().numpy()
                        ok = ok and np.array_equal(gf.reshape(len(nz), S).any(axis=1), nz)
                elif xnode is not None:
                    # the last block: it went through the last handle's GPU
                    # blocks' levels lie packed: a block holds counts/n
                    # frames of each level (fewer than B for volumes)
                    fb = w * h * bpp
                    base = (xnode["n"] - 1) * (xnode["counts"][L] // xnode["n"]) * fb
                    got = xnode["levels"][L][base + k * fb:base + (k + 1) * fb].cpu().numpy()
                    ok = ok and np.array_equal(got, r.view(np.uint8).reshape(-1))
                else:
                    got = outs[L][k * w * h * bpp:(k + 1) * w * h * bpp].cpu().numpy()
                    ok = ok and np.array_equal(got, r.view(np.uint8).reshape(-1))
                emitted[L] += 1
        check = ("bit-exact" if ok else "MISMATCH") + f" ({nchk} frame(s) vs oracle)"

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # Kernel timing with HIP events on the launch stream.  Default: one event
    # before the first launch of the timed region and one after the last, so
    # the launches run back to back as in production and the average launch
    # is span / steps — an event pair around every launch left a 12 us gap
    # between kernels (2.7% at the headline; profiles/r04/bench/).  In
    # --xgmi-scatter mode (and with --per-launch-events) every launch gets
    # its own pair, so the kernel's time sits apart from the p2p batches.
    per_launch = xgmi or args.per_launch_events
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4))
           for _ in range(args.steps if per_launch else 1)]

    def timed_step(i):
        if per_launch:
            step(evs[i])
            return
        if i == 0:
            evs[0][1].record(stream)
        step()
        if i == args.steps - 1:
            evs[0][2].record(stream)

    elapsed = timed_region(timed_step, args.steps, dist, torch.cuda.synchronize)
    xgmi_node = None
    if node_devices is not None:
        # the node's span per step (rank 0), then the kernel alone: the
        # plain local batch back to back, as in the N=1 line
        if xnode is not None:
            span_ms = evs[0][1].elapsed_time(evs[0][2]) / args.steps
            ND = xnode["n"]
            remote = sum(1 for d in node_devices if d != device) if not args.stage_all else ND
            # per remote block: its frames pulled, its levels pushed back
            moved = remote * sum(o.numel() for o in [d_in] + outs[1:])
            xgmi_node = {"ms_per_step": round(span_ms, 4), "devices": node_devices,
                         "frames_per_step": ND * B,
                         "bytes_moved_per_step": moved,
                         "moved_GBps": round(moved / (span_ms * 1e-3) / 1e9, 1),
                         "staged_blocks": remote,
                         "counts": xnode["counts"],
                         "path": "aqz_node_run_device_batch: rank 0's batch dealt in whole "
                                 "shard units, remote blocks pulled/pushed by hipMemcpyPeerAsync "
                                 "(xGMI DMA) through two staging slots per GPU, levels back "
                                 "in frame order"}
            if len(set(node_devices)) < len(node_devices):
                xgmi_node["rehearsal"] = (f"{len(node_devices)} handles on "
                                          f"{len(set(node_devices))} device(s): the staged "
                                          "copies stay on one GPU")
        kev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        torch.cuda.synchronize()
        kev[0].record(stream)
        for _ in range(args.steps):
            counts[:] = batch()
        kev[1].record(stream)
        torch.cuda.synchronize()
        launch_ms = [kev[0].elapsed_time(kev[1]) / args.steps]
    else:
        launch_ms = ([e[1].elapsed_time(e[2]) for e in evs] if per_launch else
                     [evs[0][1].elapsed_time(evs[0][2]) / args.steps])
    comm_ms = ([e[0].elapsed_time(e[1]) + e[2].elapsed_time(e[3]) for e in evs]
               if xgmi else None)
    dev = "cuda" if (dist is not None and dist.get_backend() == "nccl") else "cpu"
    elapsed = max_over_ranks(elapsed, dist, dev)
    # every rank's average launch (us) and p2p time (ms), gathered for the
    # N > 1 line
    rank_launch_us = [float(np.mean(launch_ms)) * 1e3]
    rank_comm_ms = [float(np.mean(comm_ms))] if xgmi else None
    if dist is not None:
        t = torch.zeros(2 * world, dtype=torch.float64, device=dev)
        t[rank] = rank_launch_us[0]
        if xgmi:
            t[world + rank] = rank_comm_ms[0]
        dist.all_reduce(t)
        rank_launch_us = [float(x) for x in t[:world].cpu()]
        if xgmi:
            rank_comm_ms = [float(x) for x in t[world:].cpu()]

    ms_per_step = elapsed / args.steps * 1e3
    value = aggregate_gpix(len(node_devices) if node_devices else world, B, W, H, args.steps,
                           elapsed)

    read_bytes, alg_bytes = algorithmic_bytes(geo, counts, B, args.method, bpp,
                                              tile=(chunk, chunk) if args.tiled else None)
    kind = ds.last_batch_kind()  # 1 fused 2-D cascade, 2 fused volume, 0 per-frame, 4 tiled
    per = {1: 4, 2: 2, 4: 4}.get(kind)  # levels per launch (kind 3: mixed, not derived)
    launches = -(-(n_levels - 1) // per) if per else None
    avg_launch_s = float(np.mean(launch_ms)) / 1e3
    achieved = alg_bytes / avg_launch_s / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None,
                "alg_bytes_per_launch": alg_bytes,
                "alg_read_bytes_per_launch": read_bytes,
                "avg_launch_us": round(avg_launch_s * 1e6, 2),
                "min_launch_us": round(min(launch_ms) * 1e3, 2) if per_launch else None,
                "launch_timing": ("HIP event pair around every launch" if per_launch else
                                  f"HIP events around the {args.steps} back-to-back launches "
                                  "of the timed region, on the launch stream"),
                "buffer_sets": n_rot}
    if n_rot > 1:
        # the same launches on one buffer set, for contrast: what the cache
        # keeps of a read set this small shows up here, not in `frac`
        kev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        torch.cuda.synchronize()
        for _ in range(3):
            batches[0]()
        kev[0].record(stream)
        for _ in range(args.steps):
            batches[0]()
        kev[1].record(stream)
        torch.cuda.synchronize()
        one_us = kev[0].elapsed_time(kev[1]) / args.steps * 1e3
        roofline["buffer_rotation"] = {
            "copies": n_rot, "bytes_per_copy": B * frame_bytes,
            "why": (f"a launch reads {read_bytes} B; {n_rot} input/output copies in turn "
                    f"keep {n_rot * read_bytes} B of reads between reuses, so the "
                    "256 MB Infinity Cache cannot serve a launch from the one before"),
            "one_buffer_set_avg_launch_us": round(one_us, 2),
            "one_buffer_set_frac": round(alg_bytes / (one_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}

    if world > 1:
        # kernel-only fractions: in --xgmi-scatter mode the p2p time is
        # reported beside them (comm_ms_per_step), never blended in
        roofline["per_rank"] = [{"rank": r, "avg_launch_us": round(u, 2),
                                 "frac": round(alg_bytes / (u * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
                                for r, u in enumerate(rank_launch_us)]
        if xgmi:
            for r, c in enumerate(rank_comm_ms):
                roofline["per_rank"][r]["comm_ms_per_step"] = round(c, 4)

    ceiling = measure_ceiling(torch, stream, d_all, read_bytes, alg_bytes - read_bytes,
                              max(5, args.steps // 2), n_rot, B * frame_bytes)
    if ceiling is not None:
        ceiling["frac_of_ceiling"] = round(achieved / ceiling["GBps"], 4)
        roofline["same_mix_ceiling"] = ceiling

    cpu_baseline = None
    e2e = None
    if rank == 0 and world == 1 and not args.no_pmc:
        # cascade_kernel or cascade_band_kernel (row bands staged in LDS)
        traffic = measure_traffic(args, "volume_kernel" if Z else "cascade_")
        if traffic is not None:
            roofline["traffic"] = traffic["bytes_per_launch"]
            roofline["traffic_detail"] = traffic
    if rank == 0 and world == 1:
        if args.cpu_seconds > 0:
            nf = min(B, 8)
            frames = d_in[:nf * frame_bytes].cpu().numpy().view(dtype).reshape(nf, H, W)
            cpu_baseline = measure_cpu(dims, geo, dtype, method, args.cpu_seconds,
                                       list(frames))
            threads = min(16, os.cpu_count() or 1)  # the box's CPU share is 16
            if threads > 1:
                cpu_baseline["parallel"] = measure_cpu_parallel(
                    dims, geo, dtype, method, max(2.0, args.cpu_seconds / 2), list(frames), threads)
        if args.e2e_frames > 0:
            e2e = measure_e2e(aqz, geo, dtype, method, args.e2e_frames, device,
                              tile=(chunk, chunk))
            e2e["pipelined"] = measure_e2e_pipelined(aqz, torch, geo, dtype, method,
                                                     d_in, min(B, 64), device)
            n_vis = torch.cuda.device_count()
            e2e["node"] = aux_leg("e2e.node", measure_e2e_node, aqz, torch, geo, dtype, method,
                                  d_in, min(B, 64),
                                  list(range(n_vis)) if n_vis > 1 else [device, device])
            if not args.tiled:
                e2e["node_device_batch"] = aux_leg(
                    "e2e.node_device_batch", measure_node_device_batch, aqz, torch, geo, dtype,
                    method, d_in, outs, counts, B, frame_bytes, device,
                    list(range(n_vis)) if n_vis > 1 else [device, device], stream, avg_launch_s)
            e2e["secondary_kernels"] = aux_leg("e2e.secondary_kernels", measure_secondary, aqz,
                                               torch, stream, d_in, W, H, dtype, chunk)
            # §8(f) row 3 end to end: c-blosc frames of device chunks vs c-blosc
            e2e["blosc_frames"] = aux_leg("e2e.blosc_frames", measure_blosc_frames, aqz, torch)
            # BASELINE configs[1]: 2048^2 uint16, 4 levels, filesystem sink
            # (in a temporary directory, or under --sink)
            import tempfile
            c2_dims = [(aqz.TIME, 0, 1, 1), (aqz.SPACE, 2048, 256, 1), (aqz.SPACE, 2048, 256, 1)]
            c2_geo = aqz.level_geometry(aqz.plan_levels(c2_dims))
            sink_root = args.sink or None
            if sink_root:
                os.makedirs(sink_root, exist_ok=True)
            with tempfile.TemporaryDirectory(dir=sink_root) as tmp:
                e2e["c2_filesystem_sink"] = aux_leg(
                    "e2e.c2_filesystem_sink", measure_e2e_sink,
                    aqz, c2_geo, np.uint16, method, args.e2e_frames, device,
                    os.path.join(tmp, "c2"))
            if args.sink:
                e2e["filesystem_sink"] = measure_e2e_sink(aqz, geo, dtype, method,
                                                          args.e2e_frames, device,
                                                          os.path.join(args.sink, "w"))

    if world > 1 and args.e2e_frames > 0:
        # host-to-host on every GPU at once: each rank over its own PCIe link
        nmulti = min(B, 32)
        e2e_multi = measure_e2e_pipelined(aqz, torch, geo, dtype, method, d_in, nmulti,
                                          device, dist, dev)
        e2e_multi["value"] = round(e2e_multi["value"] * world, 3)
        e2e_multi["pcie_GBps"] = round(e2e_multi["pcie_GBps"] * world, 1)
        e2e_multi["path"] += f", all {world} ranks at once (aggregate, max-over-ranks time)"
        e2e = {"pipelined_all_ranks": e2e_multi}
        # the library's own node sharding (aqz_node): ONE process
        # dealing host frames over all the ranks' GPUs, each over its own PCIe
        # link.  The other ranks wait on a CPU-only group meanwhile, so no
        # collective kernel spins on their GPUs.
        with stdout_to_stderr():
            cpu_group = dist.new_group(backend="gloo")
        if rank == 0:
            n_vis = torch.cuda.device_count()
            # a gloo rehearsal on a smaller box repeats ordinals, as the ranks do
            rehearsal = n_vis < world and os.environ.get("AQZ_DIST_BACKEND") == "gloo"
            if n_vis >= world or rehearsal:
                # guarded: the other ranks wait at the barrier below, so an
                # exception here must not leave rank 0 without reaching it
                e2e["node"] = aux_leg("e2e.node", measure_e2e_node, aqz, torch, geo, dtype,
                                      method, d_in, min(B, 64),
                                      [r % n_vis for r in range(world)])
                if not args.tiled:
                    # config F's shape of work: rank 0's device-resident batch
                    # dealt over every rank's GPU by peer copies (xGMI)
                    e2e["node_device_batch"] = aux_leg(
                        "e2e.node_device_batch", measure_node_device_batch, aqz, torch, geo,
                        dtype, method, d_in, outs, counts, B, frame_bytes, device,
                        [r % n_vis for r in range(world)], stream, avg_launch_s,
                        local_launch_shared=rehearsal)
                if rehearsal:
                    e2e["node"]["rehearsal"] = f"{world} handles on {n_vis} device(s)"
            else:
                e2e["node"] = {"skipped": f"{n_vis} device(s) visible to rank 0, "
                                          f"{world} needed"}
        dist.barrier(group=cpu_group)

    if rank == 0:
        metric = HEADLINE_METRIC if (args.workload == "4096x4096_u16" and not args.shape
                                     and not args.tiled) else (
            f"GPixels/s device-resident multiscale downsample, {W}x{H} "
            f"{np.dtype(dtype).name}, {n_levels} levels" +
            (f", chunk-tiled {chunk}x{chunk}" if args.tiled else ""))
        line = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "GPixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": np.dtype(dtype).name.replace("uint", "u").replace("float", "f"),
            "data": "synthetic (uniform random, seeded per rank)",
            "config": {"workload": f"{args.workload}: {W}x{H}" + (f"x{Z} volume" if Z else "")
                                   + f" {np.dtype(dtype).name}, {n_levels} levels, "
                                   f"{args.method}, device-resident batch",
                       "frames_per_step_per_gpu": B, "levels": n_levels,
                       "launches_per_step": launches,
                       "batch_path": {0: "per-frame", 1: "fused cascade",
                                      2: "fused volume",
                                      3: "batched, partly single-level",
                                      4: "fused cascade, chunk-tiled levels"}.get(kind, "?"),
                       "parallelism": (f"rank-0 batch scattered/gathered over xGMI "
                                       f"(RCCL p2p) x{world}" if xgmi else
                                       f"rank-0 batch of {len(node_devices)}x{B} frames sharded "
                                       f"over devices {node_devices} by aqz_node_run_device_batch"
                                       if node_devices else
                                       f"frame-sharded x{world}, no collective")
                                      + (f"; process group {dist.get_backend()} "
                                         f"world_size={dist.get_world_size()}"
                                         if dist is not None else ""),
                       "check": check},
            "comm_ms_per_step": (round(max(rank_comm_ms), 4) if xgmi else None),
            "xgmi_node": xgmi_node,
            # the binary that ran: its source revision and build time
            "library": aqz.lib().aqz_version().decode(),
            "roofline": roofline,
            "cpu_baseline": cpu_baseline,
            "e2e": e2e,
        }
        n_vis = torch.cuda.device_count()
        if world > 1 and n_vis < world:
            # ranks share GPUs (a gloo rehearsal on a smaller box): not a
            # world-GPU result, whatever n_gpus says
            line["rehearsal"] = (f"{world} ranks on {n_vis} visible device(s): "
                                 f"not a {world}-GPU measurement")
        print(json.dumps(line), flush=True)
    if xnode is not None:
        xnode["node"].close()
    ds.close()
    if dist:
        dist.destroy_process_group()


def measure_secondary(aqz, torch, stream, d_in, W, H, dtype, chunk, reps=20):
    """§8(f) kernels on level-0 frames, timed with HIP events on the launch
    stream: chunk tiling (aqz_tile_frame_device, chunk x chunk tiles),
    transpose_frame (aqz_transpose_frame_device), the blosc filters over the
    frame's chunks and crc32c over index-table-sized buffers.  The tiling,
    transpose and filters move 2 * frame_bytes algorithmic bytes (read once,
    write once in the new order; the tiling's overhang is zero at these
    sizes); crc32c reads its bytes once.  Two timings per kernel:
      avg_launch_us : one event pair per launch on one frame (the frame stays
                      in the 256 MiB Infinity Cache; includes launch latency)
      stream_*      : `reps` launches back to back over successive frames of
                      the resident batch, one event pair around all of them
                      (reads from HBM, launch gaps hidden: a streaming caller)
    CPU columns time the oracle's restatements on one core (transpose_frame
    as the reference writes it)."""
    import oracle as orc_mod  # cpu column only
    bpp = np.dtype(dtype).itemsize
    fb = W * H * bpp
    nfr = max(1, d_in.numel() // fb)
    ntx, nty = -(-W // chunk), -(-H // chunk)
    tiles = torch.empty(ntx * nty * chunk * chunk * bpp, dtype=torch.uint8, device="cuda")
    nz = torch.empty(ntx * nty, dtype=torch.int32, device="cuda")
    tout = torch.empty(fb, dtype=torch.uint8, device="cuda")
    sptr = stream.cuda_stream
    base = d_in.data_ptr()
    res = {}

    def timed(name, launch, alg_bytes):
        # launch(src_ptr, i): i-th launch reading frame src_ptr
        for i in range(3):
            launch(base, i)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(reps)]
        for i, (a, b) in enumerate(ev):
            a.record(stream)
            launch(base, i)
            b.record(stream)
        torch.cuda.synchronize()
        us = float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e3
        gbs = alg_bytes / (us * 1e-6) / 1e9
        res[name] = {"avg_launch_us": round(us, 2), "alg_bytes": alg_bytes,
                     "achieved_GBps": round(gbs, 1),
                     "frac": round(gbs / HBM_PEAK_GBS, 4)}
        n = max(reps, min(4 * nfr, 256))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for i in range(n):
            launch(base + (i % nfr) * fb, i)
        b.record(stream)
        torch.cuda.synchronize()
        sus = a.elapsed_time(b) * 1e3 / n
        sgbs = alg_bytes / (sus * 1e-6) / 1e9
        res[name].update({"stream_us_per_frame": round(sus, 2),
                          "stream_GBps": round(sgbs, 1),
                          "stream_frac": round(sgbs / HBM_PEAK_GBS, 4)})

    slice_flags = torch.empty(ntx * nty * aqz.tile_slices(chunk, chunk), dtype=torch.uint8,
                              device="cuda")
    timed("tile_kernel", lambda src, i: aqz.tile_frame_device_sliced(
        dtype, src, W, H, chunk, chunk, tiles.data_ptr(), slice_flags.data_ptr(), sptr),
        fb + ntx * nty * chunk * chunk * bpp)
    timed("tile_kernel_u32_flags_with_memset", lambda src, i: aqz.tile_frame_device(
        dtype, src, W, H, chunk, chunk, tiles.data_ptr(), nz.data_ptr(), sptr),
        fb + ntx * nty * chunk * chunk * bpp)
    timed("transpose_kernel", lambda src, i: aqz.transpose_frame_device(
        dtype, src, H, W, tout.data_ptr(), sptr), 2 * fb)
    # size-matched ceiling: a D2D copy of the same frame (read + write fb)
    timed("d2d_copy_same_bytes", lambda src, i: tout.copy_(
        d_in[src - base:src - base + fb]), 2 * fb)
    # §8(f) row 3: blosc filters over the frame as chunk-depth-1 chunks
    # (chunk x chunk tiles, 64 KiB blocks), one launch for all chunks
    cbytes = chunk * chunk * bpp
    nchunks = fb // cbytes
    for name, mode in (("blosc_shuffle", aqz.SHUFFLE), ("blosc_bitshuffle", aqz.BITSHUFFLE)):
        timed(name, lambda src, i, mode=mode: aqz.blosc_filter_device(
            mode, bpp, 65536, src, cbytes, nchunks, tout.data_ptr(), sptr), 2 * nchunks * cbytes)
    # §8(f) row 4: crc32c of 64 shard index tables of 4096 chunks (64 KiB each)
    # (its own rotation: 4 MiB of tables per launch, whatever the frame size)
    crcs = torch.empty(64, dtype=torch.int32, device="cuda")
    tb = 64 * (4096 * 16 + 4)
    ncrc = max(1, d_in.numel() // tb)
    timed("crc32c_64_index_tables", lambda src, i: aqz.crc32c_device(
        base + (i % ncrc) * tb, 4096 * 16, 4096 * 16 + 4, 64, crcs.data_ptr(), sptr),
        64 * 4096 * 16)
    # and 1024 tables of 64 chunks (1 KiB each): one workgroup per table,
    # no preset fill
    crcs_small = torch.empty(1024, dtype=torch.int32, device="cuda")
    tbs = 1024 * (64 * 16 + 4)
    ncrcs = max(1, d_in.numel() // tbs)
    timed("crc32c_1024_small_index_tables", lambda src, i: aqz.crc32c_device(
        base + (i % ncrcs) * tbs, 64 * 16, 64 * 16 + 4, 1024, crcs_small.data_ptr(), sptr),
        1024 * 64 * 16)
    raw = d_in[:cbytes * 16].cpu().numpy()
    t0 = time.perf_counter()
    for k in range(16):
        orc_mod.blosc_filter(raw[k * cbytes:(k + 1) * cbytes], aqz.BITSHUFFLE, bpp, 65536)
    res["blosc_bitshuffle"]["cpu_oracle_ms_per_frame"] = round(
        (time.perf_counter() - t0) * 1e3 * nchunks / 16, 2)
    frame = d_in[:fb].cpu().numpy().view(dtype).reshape(H, W)
    t0 = time.perf_counter()
    orc_mod.transpose_frame(frame)
    res["transpose_kernel"]["cpu_reference_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    return res


def measure_blosc_frames(aqz, torch, threads=16, n_chunks=256, reps=5):
    """compress_in_place (zarr.common.cpp:106-137) on one headline frame's
    level-0 chunks (256 x 256x256 u16; smooth synthetic image + noise, since
    the uniform bench input is incompressible): aqz_blosc_compress_device
    from device-resident chunks against c-blosc itself on `threads` C
    threads from host-resident chunks (oracle/libblosc_cpu.so, the CPU leg),
    lz4 clevel 1 with byte shuffle.  Frames are checked byte-identical."""
    import ctypes
    import blosc_ref  # checker / CPU leg only
    if not blosc_ref.available():
        return None
    rng = np.random.default_rng(5)
    yy, xx = np.mgrid[0:256, 0:256]
    host = np.empty((n_chunks, 256, 256), np.uint16)
    for k in range(n_chunks):
        host[k] = (2000 + 500 * np.sin((xx + 13 * k) / 17.0) * np.cos((yy - 5 * k) / 23.0)
                   + rng.normal(0, 4, (256, 256))).astype(np.uint16)
    raw = host.view(np.uint8).reshape(-1)
    nb = 256 * 256 * 2
    stride = nb + aqz.BLOSC_MAX_OVERHEAD
    d = torch.from_numpy(raw.copy()).to("cuda")
    torch.cuda.synchronize()
    ctx = aqz.BloscContext(torch.cuda.current_device(), threads)
    dst = np.empty(n_chunks * stride, np.uint8)
    sizes = ctx.compress_device(1, aqz.SHUFFLE, 2, "lz4", d.data_ptr(), nb, n_chunks,
                                host_dst=dst, dst_stride=stride)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.compress_device(1, aqz.SHUFFLE, 2, "lz4", d.data_ptr(), nb, n_chunks,
                            host_dst=dst, dst_stride=stride)
        ts.append(time.perf_counter() - t0)
    ctx.close()
    cpu = ctypes.CDLL(os.path.join(ROOT, "oracle", "libblosc_cpu.so"))
    cpu.cblosc_compress_chunks.restype = ctypes.c_double
    cpu.cblosc_compress_chunks.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
    cdst = np.empty(n_chunks * stride, np.uint8)
    csz = (ctypes.c_size_t * n_chunks)()
    t16 = cpu.cblosc_compress_chunks(raw.ctypes.data, nb, n_chunks, 1, 1, 2, b"lz4", threads,
                                     cdst.ctypes.data, stride, csz, reps)
    t1 = cpu.cblosc_compress_chunks(raw.ctypes.data, nb, n_chunks, 1, 1, 2, b"lz4", 1,
                                    cdst.ctypes.data, stride, csz, 1)
    same = all(sizes[k] == csz[k] and np.array_equal(dst[k * stride:k * stride + sizes[k]],
                                                     cdst[k * stride:k * stride + csz[k]])
               for k in range(n_chunks))
    return {"chunks": n_chunks, "chunk_bytes": nb, "codec": "lz4 clevel 1 shuffle",
            "ratio": round(sum(sizes) / raw.size, 4), "threads": threads,
            "aqz_device_chunks_ms": round(min(ts) * 1e3, 3),
            "cblosc_host_chunks_ms": round(t16 * 1e3, 3),
            "cblosc_1thread_ms": round(t1 * 1e3, 3),
            "frames_identical_to_cblosc": bool(same),
            "cblosc_version": blosc_ref.version()}


def rotation_copies(in_bytes: int, method: str, volume: bool, rotate_mib: int) -> int:
    """Buffer sets the timed launches take in turn: enough that the bytes a
    launch reads (Decimate reads every other row, and for volumes every
    other plane too), summed over the sets, reach `rotate_mib` MiB.  Round 5
    (DESIGN.md §11.11): volume Decimate reads 128 MiB per launch, which the
    256 MB Infinity Cache held from one launch to the next; at four volumes
    per launch the same kernel ran 30% slower per volume."""
    if rotate_mib <= 0 or in_bytes <= 0:
        return 1
    read = in_bytes // (4 if volume else 2) if method == "decimate" else in_bytes
    return max(1, min(64, -(-(rotate_mib << 20) // max(1, read))))


def measure_ceiling(torch, stream, d_in, read_bytes, write_bytes, reps, n_rot=1,
                    copy_bytes=0):
    """Measured HBM ceiling for the kernel's own byte mix (tools/hbm_probe.hip):
    a contiguous stream reading the same input buffer and writing (non-
    temporal stores) in the nearest of the ratios 12:4, 13:3, 14:2, 10:6, 9:7
    (4 KiB blocks per workgroup), plus a read-only pass, timed with HIP events
    on the launch stream.  Round 5: each pass runs with nontemporal and with
    plain loads and the faster counts (plain loads beat nontemporal ones on
    the volume Decimate launch), so the ceiling is the best
    of both policies.  With `n_rot` buffer sets (rotation_copies) the passes
    take the input copies `copy_bytes` apart and as many output regions in
    turn, as the timed launches do.  A measurement aid, not product code:
    skipped (None) if the probe library was not built."""
    import ctypes
    path = os.path.join(ROOT, "tools", "libaqz_hbm_probe.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.aqz_hbm_probe_ld.restype = ctypes.c_int
    lib.aqz_hbm_probe_ld.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    frac_r = read_bytes / max(1, read_bytes + write_bytes)
    rd, wr = min(((12, 4), (13, 3), (14, 2), (10, 6), (9, 7)), key=lambda m: abs(m[0] / 16 - frac_r))
    dst_bytes = (read_bytes // rd * wr + 4096 + 4095) // 4096 * 4096
    dst = torch.empty(n_rot * dst_bytes, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(16, dtype=torch.uint8, device="cuda")
    out = {}
    for name, (r, w) in (("GBps", (rd, wr)), ("read_only_GBps", (16, 0))):
        best = {}
        for nt in (1, 0):
            moved = ctypes.c_uint64(0)
            turn = [0]

            def go():
                k = turn[0] % n_rot
                turn[0] += 1
                rc = lib.aqz_hbm_probe_ld(d_in.data_ptr() + k * copy_bytes, read_bytes,
                                          dst.data_ptr() + k * dst_bytes,
                                          sink.data_ptr(), r, w, nt, stream.cuda_stream,
                                          ctypes.byref(moved))
                if rc != 0:
                    raise RuntimeError(f"aqz_hbm_probe_ld failed: {rc}")
            for _ in range(3):
                go()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(reps)]
            for a, b in ev:
                a.record(stream)
                go()
                b.record(stream)
            torch.cuda.synchronize()
            us = float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e3
            best["nt" if nt else "plain"] = round(moved.value / (us * 1e-6) / 1e9, 1)
        out[name] = max(best.values())
        out[name + "_by_load"] = best
    out["read_write"] = f"{rd}:{wr}"
    out["buffer_sets"] = n_rot
    out["kernel"] = ("tools/hbm_probe.hip: contiguous loads (best of nt and plain) and nt "
                     "stores, one 4 KiB-block round per workgroup, same input buffer and "
                     "stream")
    return out


def measure_traffic(args, kernel):
    """HBM bytes per cascade launch from PMC counters, one counter per
    rocprofv3 pass (MI355X_MICROARCH.md §HBM / rocprofv3 PMC slots):
      FETCH_SIZE (KiB) x 1024 x 2  — gfx950 counts half of wide streaming reads
      WRITE_SIZE (KiB) x 1024      — checked against the known output bytes
    Skipped (None) when rocprofv3 is absent or bench already runs under a
    profiler."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if not exe or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="aqz_pmc_", dir="/tmp")
        cmd = [exe, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc",
               "--", sys.executable, os.path.abspath(__file__), "--pmc-child",
               "--workload", args.workload, "--batch", str(args.batch),
               "--method", args.method, "--steps", "3", "--warmup", "1", "--no-check",
               "--rotate-mib", str(args.rotate_mib)]
        if args.tiled:
            cmd.append("--tiled")
        if args.no_flags:
            cmd.append("--no-flags")
        if args.chunk:
            cmd += ["--chunk", str(args.chunk)]
        if args.shape:
            cmd += ["--shape", args.shape]
        env = dict(os.environ, TMPDIR="/tmp")
        try:
            r = subprocess.run(cmd, env=env, capture_output=True, text=True,
                               timeout=300, cwd="/tmp")
        except subprocess.TimeoutExpired:
            return None
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not files:
            return None
        per = []
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                    per.append((int(row.get("Dispatch_Id") or len(per)),
                                float(row["Counter_Value"])))
        shutil.rmtree(d, ignore_errors=True)
        if not per:
            return None
        # the child runs 1 warm-up + 3 timed steps; a step of a deep pyramid
        # is several launches (levels 5+ chain a second one): sum per step,
        # average over the timed steps
        per = [v for _, v in sorted(per)]
        k = max(1, len(per) // 4)
        steps = [sum(per[i:i + k]) for i in range(0, len(per) - len(per) % k, k)]
        vals[counter] = float(np.mean(steps[1:] if len(steps) > 1 else steps))
    fetch = vals["FETCH_SIZE"] * 1024 * 2
    write = vals["WRITE_SIZE"] * 1024
    return {"bytes_per_launch": int(fetch + write), "read_bytes": int(fetch),
            "write_bytes": int(write), "FETCH_SIZE_KiB": vals["FETCH_SIZE"],
            "WRITE_SIZE_KiB": vals["WRITE_SIZE"],
            "correction": "FETCH_SIZE x1024 x2 (gfx950 half-count), WRITE_SIZE x1024"}


def host_info():
    """CPU model and core counts of the host the CPU baseline runs on
    (BASELINE.md §4.2): `nproc` is what this process may run on (the box's
    CPU share is smaller than the machine; `os_cpu_count` is the machine)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        nproc = len(os.sched_getaffinity(0))
    except AttributeError:
        nproc = os.cpu_count()
    return {"cpu_model": model, "nproc": nproc, "os_cpu_count": os.cpu_count()}


def _cpu_impl(dims, geo, dtype, method):
    """One CPU Downsampler and its per-frame step: the REFERENCE ITSELF
    (oracle/_ref: downsampler.cpp compiled unmodified with its Release flags,
    -O3 -mavx2) where it was built, else the oracle port.  Returns
    (kind, load(frame), step(), what)."""
    import ref as ref_mod  # cpu_baseline leg: the reference, as the baseline
    n_levels = len(geo)
    if ref_mod.available():
        r = ref_mod.RefDownsampler(dims, dtype, method)
        assert r.geometry == [tuple(g) for g in geo], (r.geometry, geo)
        take = ref_mod.lib().ref_ds_take_frame

        def step():
            # add_frame, then take_frame of every level by swap, as
            # MultiscaleArray::write_multiscale_frames_ does (no copy out)
            r.add_buffered()
            for L in range(1, n_levels):
                take(r._h, L, None, 0, None)
        return ("reference", r.load_frame, step,
                "the reference's own zarr::Downsampler (oracle/_ref: acquire-zarr "
                "src/streaming/downsampler.cpp compiled unmodified, -O3 -DNDEBUG -mavx2) "
                "add_frame + take_frame of every level")
    return _port_impl(geo, dtype, method)  # where oracle/_ref was not built


def _time_cpu(kind_pref, dims, geo, dtype, method, seconds, frames):
    impl = _port_impl(geo, dtype, method) if kind_pref == "port" else \
        _cpu_impl(dims, geo, dtype, method)
    kind, load, step, what = impl
    for i in range(2):
        load(frames[i % len(frames)])
        step()
    n, el = 0, 0.0
    while el < seconds or n < 4:
        load(frames[n % len(frames)])   # outside the timed region
        t0 = time.perf_counter()
        step()
        el += time.perf_counter() - t0
        n += 1
    return kind, what, n, el


def _port_impl(geo, dtype, method):
    import oracle as orc_mod  # cpu_baseline leg: the port, for the ratio
    o = orc_mod.OracleDownsampler(geo, dtype, method)
    cur = {}

    def step():
        o.add_frame(cur["f"])
        for L in range(1, len(geo)):
            o.take_frame(L)
    return ("port", lambda f: cur.__setitem__("f", f), step,
            "oracle/ds_oracle.c Downsampler add_frame+take_frame (-O3 -mavx2)")


def measure_cpu(dims, geo, dtype, method, seconds, frames):
    """The CPU baseline on one core over a bounded sample of the same
    workload: frame after frame (planes in Z order for volumes) until
    `seconds` of CPU work have been timed.  The reference itself
    (kind "reference") where oracle/_ref was built; the oracle port is timed
    beside it for SURVEY §8(d)'s port-vs-reference ratio."""
    W, H, _ = geo[0]
    kind, what, n, el = _time_cpu("ref", dims, geo, dtype, method, seconds, frames)
    out = {"value": round(n * W * H / el / 1e9, 4), "unit": "GPixels/s", "cores": 1,
           "kind": kind, **host_info(),
           "sample": f"{n} frames of {W}x{H} {np.dtype(dtype).name} through the "
                     f"{len(geo)}-level pyramid ({el:.1f} s timed): {what}, single thread",
           "ms_per_frame": round(el / n * 1e3, 3)}
    if kind == "reference":
        _, pwhat, pn, pel = _time_cpu("port", dims, geo, dtype, method,
                                      max(2.0, seconds / 3), frames)
        out["port"] = {"value": round(pn * W * H / pel / 1e9, 4),
                       "ms_per_frame": round(pel / pn * 1e3, 3),
                       "sample": f"{pn} frames ({pel:.1f} s timed): {pwhat}"}
        out["reference_over_port_time"] = round((el / n) / (pel / pn), 3)
    return out


def measure_cpu_parallel(dims, geo, dtype, method, seconds, frames, threads):
    """Upper-bound CPU figure: `threads` host threads, each driving its own
    Downsampler (the reference where built, else the port) over its own
    frames (independent streams, sharded like the GPUs shard frames).
    ctypes releases the GIL inside the C calls, so the threads run
    concurrently.  The reference itself runs one downsampler per stream on
    one consumer thread (zarr.stream.cpp:1616-1630); this is what a host with
    `threads` free cores could do with as many streams."""
    import threading
    W, H, _ = geo[0]
    counts = [0] * threads
    start = threading.Barrier(threads + 1, timeout=120)  # a failed worker breaks it
    stop = threading.Event()
    kinds = [None] * threads

    def worker(k):
        kind, load, step, _ = _cpu_impl(dims, geo, dtype, method)
        kinds[k] = kind
        load(frames[k % len(frames)])
        for i in range(2):  # warm
            step()
        start.wait()
        n = 0
        while not stop.is_set():
            step()
            n += 1
        counts[k] = n

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    for t in ts:
        t.start()
    start.wait()
    t0 = time.perf_counter()
    time.sleep(seconds)
    stop.set()
    for t in ts:
        t.join()
    el = time.perf_counter() - t0
    n = sum(counts)
    return {"value": round(n * W * H / el / 1e9, 4), "unit": "GPixels/s", "cores": threads,
            "kind": kinds[0],
            "sample": f"{n} frames of {W}x{H} {np.dtype(dtype).name} over {threads} "
                      f"threads, one Downsampler each ({el:.1f} s)"}


def measure_e2e(aqz, geo, dtype, method, n_frames, device, tile=None):
    """Streaming drop-in path: pageable host frame -> pinned staging -> H2D ->
    fused kernels -> D2H of levels 1..N -> take_frame copies."""
    W, H, _ = geo[0]
    rng = np.random.default_rng(3)
    if np.dtype(dtype).kind == "f":
        frames = [rng.uniform(-1000, 1000, (H, W)).astype(dtype) for _ in range(4)]
    else:
        frames = [rng.integers(0, np.iinfo(dtype).max, (H, W), dtype=dtype,
                               endpoint=True) for _ in range(4)]
    ds = aqz.Downsampler(geo, dtype, method, device=device)
    for i in range(3):
        ds.add_frame(frames[i % 4])
        for L in range(1, len(geo)):
            ds.take_frame(L)
    t0 = time.perf_counter()
    for i in range(n_frames):
        ds.add_frame(frames[i % 4])
        for L in range(1, len(geo)):
            ds.take_frame(L)
    el = time.perf_counter() - t0
    res = {"value": round(n_frames * W * H / el / 1e9, 3), "unit": "GPixels/s",
           "ms_per_frame": round(el / n_frames * 1e3, 3),
           "path": "add_frame(host) + take_frame(all levels), synchronous, 1 GPU",
           "frames": n_frames}
    if tile:
        # same loop with the chunk-tiled take: levels
        # are tiled on the GPU behind the pyramid and arrive tile-major with
        # the zero scan done
        for L in range(1, len(geo)):
            ds.set_level_tiling(L, tile[0], tile[1])
        t0 = time.perf_counter()
        for i in range(n_frames):
            ds.add_frame(frames[i % 4])
            for L in range(1, len(geo)):
                ds.take_frame_tiled(L, tile[0], tile[1])
        el = time.perf_counter() - t0
        res["tiled_take_ms_per_frame"] = round(el / n_frames * 1e3, 3)
        res["tile"] = list(tile)
        res["tiled_one_pass_runs"] = ds.stream_tiled_runs()
        if (W, H, np.dtype(dtype), tuple(tile)) == (4096, 4096, np.dtype(np.uint16), (256, 256)):
            ds.close()  # the probe's handle takes its place on this GPU
            res["async_overlap"] = aux_leg("e2e.async_overlap", measure_async_overlap, device)
            return res
    ds.close()
    return res


def measure_async_overlap(device, frames=24):
    """SURVEY §8(f) row 1 as the patched MultiscaleArray::write_frame runs it
    (acquire-zarr-hip.patch; multiscale.array.cpp:57-74,291-325), timed by the
    C++ caller tools/write_frame_probe.cpp (the reference's
    Array::write_frame_to_chunks_ restated: level 0 chunked by an OpenMP loop
    of row copies with the zero scan, array.cpp:507-622, chunk.cpp:17-58),
    run as a child process on this GPU: per 4096^2 u16 frame, 5 levels, 256^2
    chunks.  `sync` is the reference's order (host-tile level 0, add_frame,
    take every level); `async` starts the add first and tiles level 0 while
    the frame crosses PCIe; `async_take` also runs the level takes in the
    add's background job.  The parts alone: host_tile, h2d_pageable (upload
    of a pageable frame) and gpu_side (everything but the host tiling); the
    ideal overlap is the larger of host_tile and gpu_side.  Bit-exactness of
    these call orders is the GPU tests' (tests/test_gpu_adapter.py overlap /
    double / asyncsync modes), not this timing's."""
    import subprocess
    probe = os.path.join(ROOT, "tools", "write_frame_probe")
    if not os.path.exists(probe):
        return {"skipped": "tools/write_frame_probe not built (make -C acquire-zarr_amd probe)"}
    env = dict(os.environ, AQZ_GPU_DEVICE=str(device))
    r = subprocess.run([probe, str(frames), "2"], capture_output=True, text=True, env=env,
                       timeout=300)
    if r.returncode != 0:
        return {"error": f"write_frame_probe exit {r.returncode}: {r.stderr.strip()[-300:]}"}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    ms = d["ms_per_frame"]
    ideal = max(ms["host_tile"], ms["gpu_side"])
    return {"sequential_ms_per_frame": ms["sync"],
            "async_overlap_ms_per_frame": ms["async"],
            "async_take_ms_per_frame": ms["async_take"],
            "host_l0_tiling_ms_per_frame": ms["host_tile"],
            "h2d_pageable_ms_per_frame": ms["h2d_pageable"],
            "gpu_side_ms_per_frame": ms["gpu_side"],
            "ideal_overlap_ms_per_frame": ideal,
            "async_over_ideal": round(ms["async"] / ideal, 3),
            "async_take_over_ideal": round(ms["async_take"] / ideal, 3),
            "async_phases_ms": d["async_phases_ms"],
            "gpu_tiled_ms_per_frame": ms["gpu_tiled"],
            "async_one_thread_fewer_ms_per_frame": ms.get("async_one_thread_fewer"),
            "host_tile_one_thread_fewer_ms_per_frame": ms.get("host_tile_one_thread_fewer"),
            "omp_threads": d["omp_threads"], "frames": frames,
            "path": "tools/write_frame_probe (C++ caller, OpenMP level-0 chunking): "
                    "add_frame_async; level 0 chunked on the host; wait; tiled takes"}


def _fs_type(path):
    """Filesystem type holding `path` (the longest /proc/mounts prefix)."""
    best, kind = "", "?"
    try:
        real = os.path.realpath(path)
        with open("/proc/mounts") as f:
            for line in f:
                parts = line.split()
                mnt = parts[1]
                if (real == mnt or real.startswith(mnt.rstrip("/") + "/")) and len(mnt) > len(best):
                    best, kind = mnt, parts[2]
    except OSError:
        pass
    return kind


def measure_e2e_sink(aqz, geo, dtype, method, n_frames, device, sink_dir):
    """Streaming drop-in path into a filesystem sink (BASELINE configs[1]'s
    "filesystem sink"): per frame add_frame + take_frame of every level, the
    frame itself and each level frame handed to writer threads that append
    them to <sink_dir>/level_<L>.raw (the reference's sink writes on pool
    threads, array.cpp:664-811).  Timed to the last byte written and
    fsync'd.  Raw level files stand in for the Zarr store: no chunking,
    compression or metadata — the acquire-zarr library around the
    downsampler (minio-cpp, crc32c) cannot be built here."""
    import concurrent.futures as cf
    import shutil
    W, H, _ = geo[0]
    os.makedirs(sink_dir, exist_ok=True)
    rng = np.random.default_rng(4)
    if np.dtype(dtype).kind == "f":
        frames = [rng.uniform(-1000, 1000, (H, W)).astype(dtype) for _ in range(4)]
    else:
        frames = [rng.integers(0, np.iinfo(dtype).max, (H, W), dtype=dtype,
                               endpoint=True) for _ in range(4)]
    files = {L: open(os.path.join(sink_dir, f"level_{L}.raw"), "wb")
             for L in range(len(geo))}
    ds = aqz.Downsampler(geo, dtype, method, device=device)
    for i in range(2):  # warm: allocations, first launches
        ds.add_frame(frames[i])
        for L in range(1, len(geo)):
            ds.take_frame(L)
    written = 0
    # one writer thread per level file: each file's frames land in order
    pools = {L: cf.ThreadPoolExecutor(max_workers=1) for L in files}
    futs = []
    t0 = time.perf_counter()
    for i in range(n_frames):
        f0 = frames[i % 4]
        ds.add_frame(f0)
        futs.append(pools[0].submit(files[0].write, f0))
        written += f0.nbytes
        for L in range(1, len(geo)):
            f = ds.take_frame(L)
            if f is not None:
                futs.append(pools[L].submit(files[L].write, f))
                written += f.nbytes
    for fu in futs:
        fu.result()
    for fh in files.values():
        fh.flush()
        os.fsync(fh.fileno())
    el = time.perf_counter() - t0
    for p in pools.values():
        p.shutdown()
    for fh in files.values():
        fh.close()
    ds.close()
    fs = _fs_type(sink_dir)
    shutil.rmtree(sink_dir, ignore_errors=True)
    return {"value": round(n_frames * W * H / el / 1e9, 3), "unit": "GPixels/s",
            "ms_per_frame": round(el / n_frames * 1e3, 3), "frames": n_frames,
            "geometry": [list(g) for g in geo], "dtype": np.dtype(dtype).name,
            "bytes_written": written, "sink_fs": fs,
            "writes": "raw level files (level 0 and every pyramid level), not a Zarr store",
            "path": "add_frame + take_frame(every level) + a writer thread per level -> "
                    "per-level raw files, fsync'd"}


def measure_e2e_pipelined(aqz, torch, geo, dtype, method, d_in, n, device, dist=None,
                          dev="cpu"):
    """Host-resident frames through aqz_ds_run_host_batch: pinned input and
    level buffers, upload / kernels / download overlapped in double-buffered
    groups — the PCIe-inclusive rate a caller that overlaps frames gets.
    With `dist`, every rank runs it at once (each GPU over its own PCIe link)
    between barriers and the time is the max over ranks."""
    W, H, _ = geo[0]
    bpp = np.dtype(dtype).itemsize
    src = d_in[:n * W * H * bpp].cpu().pin_memory()
    outs = [None] + [torch.empty(n * w * h * bpp, dtype=torch.uint8).pin_memory()
                     for w, h, _ in geo[1:]]
    ptrs = [0] + [o.data_ptr() for o in outs[1:]]
    ds = aqz.Downsampler(geo, dtype, method, device=device)
    ds.run_host_batch(src.data_ptr(), n, ptrs)  # warm: allocates the pipeline
    best = None
    for _ in range(3):
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        ds.run_host_batch(src.data_ptr(), n, ptrs)
        el = max_over_ranks(time.perf_counter() - t0, dist, dev)
        best = el if best is None else min(best, el)
    ds.close()
    in_bytes = n * W * H * bpp
    out_bytes = sum(o.numel() for o in outs[1:])
    return {"value": round(n * W * H / best / 1e9, 3), "unit": "GPixels/s",
            "ms_per_frame": round(best / n * 1e3, 3),
            "pcie_GBps": round((in_bytes + out_bytes) / best / 1e9, 1),
            "path": "aqz_ds_run_host_batch, pinned host in/out, "
                    f"{n} frames, H2D/kernels/D2H overlapped"}


def aux_leg(name, fn, *args, **kwargs):
    """Run one auxiliary measurement (an `e2e` sub-leg, after the timed
    region and the oracle check).  A failure there is reported in the line
    as {"error": ...}, with its traceback on stderr, rather than losing the
    line or, at N > 1, leaving the other ranks waiting at a barrier."""
    try:
        return fn(*args, **kwargs)
    except Exception as e:  # reported, never silent
        import traceback
        traceback.print_exc(file=sys.stderr)
        print(f"bench: {name} failed: {type(e).__name__}: {e}", file=sys.stderr)
        return {"error": f"{type(e).__name__}: {e}"}


def measure_node_device_batch(aqz, torch, geo, dtype, method, d_in, outs, counts, B,
                              frame_bytes, device, devices, stream, local_launch_s, reps=5,
                              local_launch_shared=False):
    """BASELINE config F's multi-GPU form through the library
    (aqz_node_run_device_batch): len(devices) copies of this
    rank's device-resident batch, on this GPU, dealt over `devices` in whole
    shard units; remote blocks are pulled and their levels pushed back by
    hipMemcpyPeerAsync (xGMI DMA), levels land in frame order.  Every block's
    levels are compared with this rank's own batch (`outs`, the timed
    kernel's output of the same frames).  The rate is set against the timed
    kernel: one GPU would take len(devices) x its launch time."""
    ND = len(devices)
    pool = torch.empty(ND * B * frame_bytes, dtype=torch.uint8, device="cuda")
    for r in range(ND):
        pool[r * B * frame_bytes:(r + 1) * B * frame_bytes].copy_(d_in[:B * frame_bytes])
    levels = [None] + [torch.empty(ND * o.numel(), dtype=torch.uint8, device="cuda")
                       for o in outs[1:]]
    torch.cuda.synchronize()
    node = aqz.Node(geo, dtype, method, devices)
    try:
        call = node.device_batch_call(pool.data_ptr(), device, ND * B,
                                      [0] + [t.data_ptr() for t in levels[1:]],
                                      stream.cuda_stream)
        got = call()  # warm: staging and streams on the remote GPUs
        torch.cuda.synchronize()
        exact = True
        for L in range(1, len(geo)):
            w, h, _ = geo[L]
            nb = counts[L] * w * h * np.dtype(dtype).itemsize
            exact = exact and got[L] == ND * counts[L]
            # the node packs each block's level frames densely: block r's
            # start at r * nb (nb < outs[L]'s size for volumes)
            for r in range(ND):
                exact = exact and bool(torch.equal(levels[L][r * nb:(r + 1) * nb],
                                                   outs[L][:nb]))
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record(stream)
        for _ in range(reps):
            call()
        ev[1].record(stream)
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
    finally:
        node.close()
    W, H, _ = geo[0]
    # the one-GPU reference time is this rank's own launch time from the
    # main region; where handles (or ranks) share a device that time was
    # itself slowed by the sharing, so no speed-up is reported
    shared = len(set(devices)) < len(devices) or local_launch_shared
    one_gpu_ms = None if shared else ND * local_launch_s * 1e3
    out = {"value": round(ND * B * W * H / (ms * 1e-3) / 1e9, 3), "unit": "GPixels/s",
           "ms_per_call": round(ms, 4), "frames_per_call": ND * B, "devices": list(devices),
           "one_gpu_ms_same_frames": None if one_gpu_ms is None else round(one_gpu_ms, 4),
           "speedup_vs_one_gpu": None if one_gpu_ms is None else round(one_gpu_ms / ms, 3),
           "check": ("bit-exact" if exact else "MISMATCH") +
                    f" (all {ND} blocks vs this rank's own batch)",
           "path": "aqz_node_run_device_batch: this GPU's batch dealt in whole shard units, "
                   "remote blocks pulled and levels pushed by hipMemcpyPeerAsync (xGMI DMA) "
                   "through two staging slots per GPU, levels in frame order"}
    if len(set(devices)) < len(devices):
        out["rehearsal"] = (f"{len(devices)} handles on {len(set(devices))} device(s): "
                            "blocks on the batch's own GPU run in place, one after "
                            "another, so no speed-up is possible")
    return out


def measure_e2e_node(aqz, torch, geo, dtype, method, d_in, n, devices):
    """Host-resident frames sharded over `devices` by the library itself
    (aqz_node_run_host_batch): one handle per entry, each
    running the pipelined host batch on its block of whole shard units in its
    own host thread, levels written back in frame-id order.  On a one-GPU box
    the entries repeat ordinal 0 (two pipelines sharing one PCIe link), so
    the rate shows the dealing's overhead, not a multi-GPU speed-up."""
    W, H, _ = geo[0]
    bpp = np.dtype(dtype).itemsize
    node = aqz.Node(geo, dtype, method, devices)
    n -= n % node.unit
    src = d_in[:n * W * H * bpp].cpu().pin_memory()
    outs = [None] + [torch.empty(n * w * h * bpp, dtype=torch.uint8).pin_memory()
                     for w, h, _ in geo[1:]]
    ptrs = [0] + [o.data_ptr() for o in outs[1:]]
    node.run_host_batch(src.data_ptr(), n, ptrs)  # warm: allocates the pipelines
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        node.run_host_batch(src.data_ptr(), n, ptrs)
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    # the streaming form: one pageable frame per call, as the frame queue
    # hands them over, levels taken whenever ready, then flushed
    host = src.numpy().view(dtype).reshape(n, H, W)
    frames = [np.array(host[k]) for k in range(min(n, 32))]
    levels = range(1, len(geo))

    def stream():
        for f in frames:
            node.add_frame(f)
            for L in levels:
                while node.take_frame(L) is not None:
                    pass
        node.flush()
        for L in levels:
            while node.take_frame(L) is not None:
                pass
    stream()  # warm
    sbest = None
    for _ in range(3):
        t0 = time.perf_counter()
        stream()
        el = time.perf_counter() - t0
        sbest = el if sbest is None else min(sbest, el)

    # the drop-in's node mode (integration/src/streaming/downsampler.hip.cpp
    # with $AQZ_GPU_DEVICES), the consumer side as Downsampler::release_frame
    # runs it: per frame add, no wait — the adapter keeps the frame's buffer
    # while its upload may run and hands the frame queue a spare, recycling
    # the kept buffers as aqz_node_inputs_released passes them — and take
    # every ready level; a flush and a last drain at the end
    # (MultiscaleArray::close_).  The queue's copy into its slot happens on
    # the producer thread and is not timed.  The buffers here are the frame
    # list's own (nothing rewrites them), so the bookkeeping is kept without
    # the spare allocations.
    def dropin(cycle):
        kept = collections.deque()
        spares = 0
        for k in range(len(frames)):
            f = cycle[k % len(cycle)]
            node.add_frame(f)
            released = node.inputs_released()
            while kept and kept[0][0] < released:
                kept.popleft()
                spares += 1
            kept.append((k, f))
            for L in levels:
                while node.take_frame(L) is not None:
                    pass
        node.flush()
        for L in levels:
            while node.take_frame(L) is not None:
                pass
        return spares
    # over the 4 recycled frames the synchronous leg (measure_e2e) streams,
    # like for like, and over the 32 distinct ones (1 GiB, which the host's
    # caches cannot hold; slower and more variable)
    dropin(frames[:4])  # warm
    dbest = dbest32 = None
    for _ in range(3):
        t0 = time.perf_counter()
        dropin(frames[:4])
        el = time.perf_counter() - t0
        dbest = el if dbest is None else min(dbest, el)
        t0 = time.perf_counter()
        dropin(frames)
        el = time.perf_counter() - t0
        dbest32 = el if dbest32 is None else min(dbest32, el)
    node.close()
    in_bytes = n * W * H * bpp
    out_bytes = sum(o.numel() for o in outs[1:])
    return {"value": round(n * W * H / best / 1e9, 3), "unit": "GPixels/s",
            "ms_per_frame": round(best / n * 1e3, 3),
            "pcie_GBps": round((in_bytes + out_bytes) / best / 1e9, 1),
            "devices": list(devices), "shard_unit": node.unit,
            "stream_ms_per_frame": round(sbest / len(frames) * 1e3, 3),
            "dropin_ms_per_frame": round(dbest / len(frames) * 1e3, 3),
            "dropin_distinct_ms_per_frame": round(dbest32 / len(frames) * 1e3, 3),
            "dropin_path": f"per pageable frame: aqz_node_add_frame, no upload wait (the "
                           "adapter keeps the buffer, recycled by aqz_node_inputs_released), "
                           "every ready level taken; flush at the end (the drop-in's "
                           "$AQZ_GPU_DEVICES mode, consumer side, Downsampler::release_frame); "
                           f"{len(frames)} adds cycling over 4 frames as e2e.ms_per_frame "
                           f"does (dropin_distinct: {len(frames)} distinct frames)",
            "stream_path": f"aqz_node_add_frame of {len(frames)} pageable frames, every level "
                           "taken when ready, then aqz_node_flush",
            "path": f"aqz_node_run_host_batch over handles on devices {list(devices)}, "
                    f"pinned host in/out, {n} frames in blocks of whole shard units"}


if __name__ == "__main__":
    main()
