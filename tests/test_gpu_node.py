"""GPU: frame sharding inside the library (aqz_node; VERDICT r3
item 3).  Several handles on ONE GPU (devices [0, 0] and [0, 0, 0]) stand in
for a node's GPUs: the dealing, the per-handle threads and pipelines and the
in-order write-back are the same code an 8-GPU node runs.  Every level must
equal one oracle stream frame for frame — 2-D and volumes, ragged blocks
(units that do not divide evenly over the handles), batches in a row."""
import zlib

import numpy as np
import pytest

from gpu_util import assert_parity, random_frames

pytestmark = pytest.mark.gpu

SPACE, TIME = 0, 2

CASES = {
    # name: (dims, frames per batch, batches)
    "2d_1000x600": ([(TIME, 0, 1, 1), (SPACE, 600, 64, 1), (SPACE, 1000, 64, 1)], 7, 2),
    "2d_4096_u16": ([(TIME, 0, 1, 1), (SPACE, 4096, 256, 1), (SPACE, 4096, 256, 1)], 5, 1),
    "vol_z16": ([(TIME, 0, 1, 1), (SPACE, 16, 4, 1), (SPACE, 256, 64, 1), (SPACE, 200, 64, 1)],
                40, 2),
    "vol_z15_odd": ([(TIME, 0, 1, 1), (SPACE, 15, 4, 1), (SPACE, 130, 32, 1),
                     (SPACE, 99, 32, 1)], 45, 1),
}


def _host(nbytes):
    return np.empty(max(nbytes, 1), np.uint8)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0], [0] * 8], ids=["x2", "x3", "x8"])
@pytest.mark.parametrize("dtype", [np.uint16, np.float32, np.uint8], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("name", list(CASES))
def test_node_host_batch_matches_oracle(aqz, oracle, name, dtype, devices):
    dims, per_batch, batches = CASES[name]
    if name == "2d_4096_u16" and dtype != np.uint16:
        pytest.skip("headline geometry: u16")
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    method = aqz.MEAN if dtype != np.uint8 else aqz.MAX
    node = aqz.Node(geo, dtype, method, devices)
    assert node.handle_devices() == devices
    w, h, _ = geo[0]
    bpp = np.dtype(dtype).itemsize
    rng = np.random.default_rng(per_batch * 31 + len(devices))
    ref = oracle.OracleDownsampler(geo, dtype, method)
    assert per_batch % node.unit == 0
    try:
        for b in range(batches):
            frames = random_frames(rng, dtype, (per_batch, h, w))
            outs = [None] + [_host(per_batch * gw * gh * bpp) for gw, gh, _ in geo[1:]]
            counts = node.run_host_batch(frames.ctypes.data, per_batch,
                                         [0] + [o.ctypes.data for o in outs[1:]])
            want = {L: [] for L in range(1, len(geo))}
            for f in frames:
                ref.add_frame(f)
                for L in want:
                    r = ref.take_frame(L)
                    if r is not None:
                        want[L].append(r)
            for L, wl in want.items():
                gw, gh, _ = geo[L]
                assert counts[L] == len(wl), f"batch {b} level {L}"
                got = outs[L][:len(wl) * gw * gh * bpp].view(dtype).reshape(len(wl), gh, gw)
                for k, e in enumerate(wl):
                    assert_parity(got[k], e, f"{name} batch {b} L{L} frame {k}")
    finally:
        node.close()


def test_node_rejects_partial_units(aqz):
    dims = CASES["vol_z16"][0]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    node = aqz.Node(geo, np.uint16, aqz.MEAN, [0, 0])
    try:
        assert node.unit == 4
        w, h, _ = geo[0]
        frames = np.zeros((6, h, w), np.uint16)
        outs = [0] + [_host(6 * gw * gh * 2).ctypes.data for gw, gh, _ in geo[1:]]
        with pytest.raises(aqz.AqzError) as e:
            node.run_host_batch(frames.ctypes.data, 6, outs)
        assert "shard units of 4" in str(e.value)
    finally:
        node.close()


def test_node_rejects_bad_ordinal(aqz):
    geo = [(64, 64, 0), (32, 32, 0)]
    with pytest.raises(aqz.AqzError):
        aqz.Node(geo, np.uint16, aqz.MEAN, [0, 4096])


def _oracle_levels(oracle, geo, dtype, method, frames):
    ref = oracle.OracleDownsampler(geo, dtype, method)
    want = {L: [] for L in range(1, len(geo))}
    for f in frames:
        ref.add_frame(f)
        for L in want:
            r = ref.take_frame(L)
            if r is not None:
                want[L].append(r)
    return want


STREAM_CASES = {
    "2d_1000x600": ([(TIME, 0, 1, 1), (SPACE, 600, 64, 1), (SPACE, 1000, 64, 1)], 11),
    "vol_z16": ([(TIME, 0, 1, 1), (SPACE, 16, 4, 1), (SPACE, 256, 64, 1), (SPACE, 200, 64, 1)], 40),
    "vol_z15_odd": ([(TIME, 0, 1, 1), (SPACE, 15, 4, 1), (SPACE, 130, 32, 1),
                     (SPACE, 99, 32, 1)], 37),   # ends inside a stack
}


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0], [0] * 8], ids=["x2", "x3", "x8"])
@pytest.mark.parametrize("dtype", [np.uint16, np.float32], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("name", list(STREAM_CASES))
def test_node_stream_matches_oracle(aqz, oracle, name, dtype, devices):
    """aqz_node_add_frame / _take_frame / _flush: frames in flight on every
    handle, levels taken whenever ready, the rest after the flush — the same
    frames in the same order as one oracle stream."""
    dims, n = STREAM_CASES[name]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    node = aqz.Node(geo, dtype, aqz.MEAN, devices)
    rng = np.random.default_rng(n + len(devices))
    w, h, _ = geo[0]
    frames = random_frames(rng, dtype, (n, h, w))
    got = {L: [] for L in range(1, len(geo))}
    try:
        for k in range(n):
            node.add_frame(frames[k])
            for L in got:
                while (r := node.take_frame(L)) is not None:
                    got[L].append(r)
        node.flush()
        for L in got:
            while (r := node.take_frame(L)) is not None:
                got[L].append(r)
    finally:
        node.close()
    want = _oracle_levels(oracle, geo, dtype, aqz.MEAN, frames)
    for L in got:
        assert len(got[L]) == len(want[L]), f"{name} level {L}: {len(got[L])} vs {len(want[L])}"
        for k, (a, b) in enumerate(zip(got[L], want[L])):
            assert_parity(a, b, f"{name} stream L{L} frame {k}")


def test_node_stream_then_batch_then_stream(aqz, oracle):
    """A batch may follow the stream at a shard-unit boundary (the stream's
    adds are flushed first) and the stream continues after it; inside a unit
    the batch is refused."""
    dims = STREAM_CASES["vol_z16"][0]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    node = aqz.Node(geo, np.uint16, aqz.MAX, [0, 0])
    w, h, _ = geo[0]
    rng = np.random.default_rng(5)
    frames = random_frames(rng, np.uint16, (24, h, w))
    got = {L: [] for L in range(1, len(geo))}

    def drain():
        for L in got:
            while (r := node.take_frame(L)) is not None:
                got[L].append(r)
    try:
        for k in range(6):                       # 1.5 units
            node.add_frame(frames[k])
        outs = [0] + [_host(8 * gw * gh * 2).ctypes.data for gw, gh, _ in geo[1:]]
        with pytest.raises(aqz.AqzError) as e:
            node.run_host_batch(frames[6:].ctypes.data, 8, outs)
        assert "inside a shard unit" in str(e.value)
        for k in range(6, 8):                    # back on a unit boundary
            node.add_frame(frames[k])
        bufs = [None] + [_host(12 * gw * gh * 2) for gw, gh, _ in geo[1:]]
        counts = node.run_host_batch(frames[8:20].ctypes.data, 12,
                                     [0] + [b.ctypes.data for b in bufs[1:]])
        drain()                                  # the stream's frames, flushed by the batch
        drain_before = {L: len(v) for L, v in got.items()}
        for L in got:
            gw, gh, _ = geo[L]
            got[L] += list(bufs[L][:counts[L] * gw * gh * 2].view(np.uint16)
                           .reshape(counts[L], gh, gw))
        for k in range(20, 24):
            node.add_frame(frames[k])
        node.flush()
        drain()
    finally:
        node.close()
    assert drain_before is not None
    want = _oracle_levels(oracle, geo, np.uint16, aqz.MAX, frames)
    for L in got:
        assert len(got[L]) == len(want[L])
        for k, (a, b) in enumerate(zip(got[L], want[L])):
            assert_parity(a, b, f"mixed L{L} frame {k}")


def _fuzz_case(i):
    rng = np.random.default_rng(zlib.crc32(f"nodefuzz{i}".encode()))
    dtype = [np.uint8, np.uint16, np.int32, np.float32, np.float64][int(rng.integers(5))]
    method = int(rng.integers(4))
    w, h = int(rng.integers(8, 700)), int(rng.integers(4, 300))
    cx, cy = int(rng.integers(8, 128)), int(rng.integers(4, 128))
    dims = [(TIME, 0, 1, 1)]
    if rng.random() < 0.5:                      # a Z stack
        z = int(rng.integers(2, 20))
        dims.append((SPACE, z, int(rng.integers(1, 6)), 1))
    dims += [(SPACE, h, cy, 1), (SPACE, w, cx, 1)]
    devices = [0] * int(rng.integers(1, 5))
    return dtype, method, dims, devices, rng


@pytest.mark.parametrize("i", range(24))
def test_node_fuzz(aqz, oracle, i):
    """Random 2-D and Z-stack geometries (even and odd stacks, Z halving at
    some levels only), dtypes, methods and 1-4 handles: a host batch of whole
    units, then a stream of any length, against one oracle stream."""
    dtype, method, dims, devices, rng = _fuzz_case(i)
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    if len(geo) < 2:
        pytest.skip("no level below the base")
    node = aqz.Node(geo, dtype, method, devices)
    w, h, _ = geo[0]
    n_batch = node.unit * int(rng.integers(1, 5))
    n_stream = int(rng.integers(1, 2 * node.unit + 3))
    frames = random_frames(rng, dtype, (n_batch + n_stream, h, w))
    bpp = np.dtype(dtype).itemsize
    got = {L: [] for L in range(1, len(geo))}
    try:
        bufs = [None] + [_host(n_batch * gw * gh * bpp) for gw, gh, _ in geo[1:]]
        counts = node.run_host_batch(frames[:n_batch].ctypes.data, n_batch,
                                     [0] + [b.ctypes.data for b in bufs[1:]])
        for L in got:
            gw, gh, _ = geo[L]
            got[L] += list(bufs[L][:counts[L] * gw * gh * bpp].view(dtype)
                           .reshape(counts[L], gh, gw))
        for k in range(n_batch, n_batch + n_stream):
            node.add_frame(frames[k])
            if rng.random() < 0.5:
                for L in got:
                    while (r := node.take_frame(L)) is not None:
                        got[L].append(r)
        node.flush()
        for L in got:
            while (r := node.take_frame(L)) is not None:
                got[L].append(r)
    finally:
        node.close()
    want = _oracle_levels(oracle, geo, dtype, method, frames)
    for L in got:
        assert len(got[L]) == len(want[L]), (i, dims, devices, L)
        for k, (a, b) in enumerate(zip(got[L], want[L])):
            assert_parity(a, b, f"fuzz {i} {dims} L{L} frame {k}")


def test_node_take_hands_out_finished_adds_early(aqz, oracle):
    """aqz_node_take_frame settles, without waiting, every add whose
    background job has finished (aqz_ds_poll), so a frame's levels come out
    before its handle is used again — here without any later add or flush."""
    import time
    dims = STREAM_CASES["2d_1000x600"][0]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    node = aqz.Node(geo, np.uint16, aqz.MEAN, [0, 0, 0])
    w, h, _ = geo[0]
    frames = random_frames(np.random.default_rng(9), np.uint16, (2, h, w))
    try:
        for f in frames:
            node.add_frame(f)
        got = {L: [] for L in range(1, len(geo))}
        deadline = time.monotonic() + 20
        while any(len(v) < 2 for v in got.values()) and time.monotonic() < deadline:
            for L in got:
                while (r := node.take_frame(L)) is not None:
                    got[L].append(r)
            time.sleep(0.001)
        assert all(len(v) == 2 for v in got.values()), {L: len(v) for L, v in got.items()}
        node.flush()
        for L in got:
            assert node.take_frame(L) is None
    finally:
        node.close()
    want = _oracle_levels(oracle, geo, np.uint16, aqz.MEAN, frames)
    for L in got:
        for k, (a, b) in enumerate(zip(got[L], want[L])):
            assert_parity(a, b, f"early L{L} frame {k}")


def test_poll_reports_the_async_job(aqz):
    """aqz_ds_poll: done with nothing pending, done again once the add
    finishes, and it leaves the job's status to aqz_ds_wait."""
    import time
    geo = [(256, 256, 1), (128, 128, 1)]
    ds = aqz.Downsampler(geo, np.uint16, aqz.MEAN)
    try:
        assert ds.poll()
        frame = np.arange(256 * 256, dtype=np.uint16).reshape(256, 256)
        ds.add_frame_async(frame)
        deadline = time.monotonic() + 20
        while not ds.poll() and time.monotonic() < deadline:
            time.sleep(0.001)
        assert ds.poll()
        ds.wait()
        assert ds.take_frame(1) is not None
    finally:
        ds.close()


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]], ids=["x2", "x3"])
def test_node_inputs_released_lets_buffers_recycle(aqz, oracle, devices):
    """The drop-in's node mode without upload waits (Downsampler::
    release_frame): a frame buffer goes back to the producer as soon as
    aqz_node_inputs_released passes its index, and is overwritten with a
    later frame while other frames are still in flight.  The count is a
    prefix that never decreases and reaches every frame after the flush, and
    the levels are still exactly one oracle stream's."""
    import collections
    dims = STREAM_CASES["vol_z16"][0]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    w, h, _ = geo[0]
    n = 40
    frames = random_frames(np.random.default_rng(17), np.uint16, (n, h, w))
    node = aqz.Node(geo, np.uint16, aqz.MEAN, devices)
    got = {L: [] for L in range(1, len(geo))}
    kept = collections.deque()  # (frame index, buffer) the node may read
    spares = []
    allocated = 0
    last = 0
    try:
        for k in range(n):
            buf = spares.pop() if spares else None
            if buf is None:
                buf = np.empty((h, w), np.uint16)
                allocated += 1
            np.copyto(buf, frames[k])   # the producer's copy into a free slot
            node.add_frame(buf)
            released = node.inputs_released()
            assert last <= released <= k + 1
            last = released
            while kept and kept[0][0] < released:
                spares.append(kept.popleft()[1])
            kept.append((k, buf))
            for L in got:
                while (r := node.take_frame(L)) is not None:
                    got[L].append(r)
        node.flush()
        assert node.inputs_released() == n
        for L in got:
            while (r := node.take_frame(L)) is not None:
                got[L].append(r)
    finally:
        node.close()
    # at most one buffer in flight per handle, plus the one being filled
    assert allocated <= len(devices) + 2, allocated
    want = _oracle_levels(oracle, geo, np.uint16, aqz.MEAN, frames)
    for L in got:
        assert len(got[L]) == len(want[L])
        for k, (a, b) in enumerate(zip(got[L], want[L])):
            assert_parity(a, b, f"recycled L{L} frame {k}")
