"""GPU: the node's device-resident batch (aqz_node_run_device_batch,
BASELINE config F "frame batches sharded across GPUs over xGMI"; VERDICT r4
item 3).

The batch and its outputs live on device 0; handles on [0, 0] / [0, 0, 0]
stand in for a node's GPUs.  Two modes:
* in place  — every handle on the batch's GPU runs its block of whole shard
  units on the caller's stream;
* staged    — AQZ_NODE_STAGE_ALL: every block takes the remote-GPU path
  (peer-copy pull into the handle's two staging slots, the pyramid on the
  handle's own stream, peer-copy push of each level back to the block's place)
  — the code a handle on another GPU runs, with $AQZ_NODE_STAGE_MB small so
  blocks move in several sub-batches and the slots are reused.
Outputs must hash to the REFERENCE-made digests of the full-size BASELINE
configs (tests/golden/reference_digests.json) and equal one oracle stream on
ragged fuzz geometries."""
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

import digest_util as du
from gpu_util import assert_parity, empty_device, launch_stream, random_frames, to_device, torch_cuda

pytestmark = pytest.mark.gpu

with open(du.GOLDEN) as f:
    GOLD = json.load(f)["configs"]

SPACE, TIME = 0, 2


class stage_mb:
    """Set $AQZ_NODE_STAGE_MB for the calls inside (read per call)."""

    def __init__(self, mb):
        self.mb = mb

    def __enter__(self):
        self.old = os.environ.get("AQZ_NODE_STAGE_MB")
        if self.mb:
            os.environ["AQZ_NODE_STAGE_MB"] = str(self.mb)

    def __exit__(self, *exc):
        if self.old is None:
            os.environ.pop("AQZ_NODE_STAGE_MB", None)
        else:
            os.environ["AQZ_NODE_STAGE_MB"] = self.old


# (config, method, devices, staged, staging MiB per slot)
DIGEST_CASES = [
    ("F_4096x4096_f32", 1, [0, 0], False, 0),
    ("F_4096x4096_f32", 1, [0, 0], True, 0),
    ("F_4096x4096_f32", 3, [0, 0, 0], True, 0),
    ("H_4096x4096_u16", 1, [0, 0], True, 0),
    ("V_1024x1024x256_u16", 1, [0, 0], False, 0),
    ("V_1024x1024x256_u16", 1, [0, 0], True, 0),
    ("V_1024x1024x256_u16", 0, [0, 0, 0], True, 16),   # 1-unit sub-batches
    ("V_1024x1024x256_u16", 3, [0] * 8, True, 40),
]


@pytest.mark.parametrize("name,method,devices,staged,mb", DIGEST_CASES,
                         ids=[f"{c}-{du.METHOD_NAMES[m]}-x{len(d)}-{'staged' if s else 'inplace'}"
                              + (f"-{mb}MB" if mb else "")
                              for c, m, d, s, mb in DIGEST_CASES])
def test_node_device_batch_matches_reference_digests(aqz, name, method, devices, staged, mb):
    torch = torch_cuda()
    dims, dtype, frames = du.CONFIGS[name]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    W, H, _ = geo[0]
    bpp = np.dtype(dtype).itemsize
    host = np.stack([du.frame(name, k, W, H, dtype) for k in range(frames)])
    d_in = to_device(host)
    outs = [None] + [empty_device(frames * w * h * bpp) for w, h, _ in geo[1:]]
    for o in outs[1:]:
        o.fill_(0xA5)
    node = aqz.Node(geo, dtype, method, devices)
    try:
        s = launch_stream()
        dev_before = torch.cuda.current_device()
        with stage_mb(mb):
            counts = node.run_device_batch(d_in.data_ptr(), 0, frames,
                                           [0] + [o.data_ptr() for o in outs[1:]], s,
                                           stage_all=staged)
        assert torch.cuda.current_device() == dev_before
        torch.cuda.synchronize()
    finally:
        node.close()
    want = GOLD[name]["methods"][du.METHOD_NAMES[method]]
    for L in range(1, len(geo)):
        w, h, _ = geo[L]
        n = counts[L]
        assert n == want[str(L)]["frames"], f"level {L} frames"
        raw = outs[L][:n * w * h * bpp].cpu().numpy()
        assert hashlib.sha256(raw.tobytes()).hexdigest() == want[str(L)]["sha256"], \
            f"level {L}"


def test_node_device_batch_f32_many_frames_equals_one_handle(aqz):
    """Config F's shape with a real batch (9 frames over 3 handles, 2 frames
    per staged sub-batch, slots reused): byte-equal to one handle's
    aqz_ds_run_device_batch, the digest-pinned path."""
    torch = torch_cuda()
    dims = du.CONFIGS["F_4096x4096_f32"][0]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    W, H, _ = geo[0]
    n = 9
    g = torch.Generator(device="cuda").manual_seed(77)
    d_in = (torch.rand(n * W * H, device="cuda", generator=g) * 2000 - 1000).view(torch.uint8)
    sizes = [n * w * h * 4 for w, h, _ in geo]
    want = [None] + [empty_device(b) for b in sizes[1:]]
    got = [None] + [empty_device(b) for b in sizes[1:]]
    s = launch_stream()
    ds = aqz.Downsampler(geo, np.float32, aqz.MEAN)
    node = aqz.Node(geo, np.float32, aqz.MEAN, [0, 0, 0])
    try:
        ds.run_device_batch(d_in.data_ptr(), n, [0] + [o.data_ptr() for o in want[1:]], s)
        with stage_mb(2 * W * H * 4 * 4 // 3 // (1 << 20) + 1):   # two frames + levels
            c = node.run_device_batch(d_in.data_ptr(), 0, n,
                                      [0] + [o.data_ptr() for o in got[1:]], s,
                                      stage_all=True)
        torch.cuda.synchronize()
    finally:
        node.close()
        ds.close()
    assert c == [n] * len(geo)
    for L in range(1, len(geo)):
        assert torch.equal(got[L], want[L]), f"level {L}"


def _fuzz(i):
    rng = np.random.default_rng(zlib.crc32(f"nodedev{i}".encode()))
    dtype = [np.uint8, np.uint16, np.int32, np.float32, np.float64][int(rng.integers(5))]
    method = int(rng.integers(4))
    w, h = int(rng.integers(16, 600)), int(rng.integers(8, 260))
    dims = [(TIME, 0, 1, 1)]
    if rng.random() < 0.5:
        dims.append((SPACE, int(rng.integers(2, 20)), int(rng.integers(1, 6)), 1))
    # chunks below half the frame: at least one level under the base
    dims += [(SPACE, h, int(rng.integers(2, h // 2 + 1)), 1),
             (SPACE, w, int(rng.integers(2, w // 2 + 1)), 1)]
    devices = [0] * int(rng.integers(1, 5))
    return dtype, method, dims, devices, bool(rng.integers(2)), rng


@pytest.mark.parametrize("i", range(20))
def test_node_device_batch_fuzz_matches_oracle(aqz, oracle, i):
    """Random 2-D and Z-stack geometries (even and odd stacks), dtypes,
    methods, 1-4 handles, in place or staged with tiny sub-batches: two
    batches in a row against one oracle stream."""
    torch = torch_cuda()
    dtype, method, dims, devices, staged, rng = _fuzz(i)
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    if len(geo) < 2:
        pytest.skip("no level below the base")
    node = aqz.Node(geo, dtype, method, devices)
    w, h, _ = geo[0]
    bpp = np.dtype(dtype).itemsize
    sizes = [int(rng.integers(1, 5)) * node.unit for _ in range(2)]
    frames = random_frames(rng, dtype, (sum(sizes), h, w))
    got = {L: [] for L in range(1, len(geo))}
    try:
        s = launch_stream()
        k0 = 0
        for nb in sizes:
            d_in = to_device(frames[k0:k0 + nb])
            outs = [None] + [empty_device(nb * gw * gh * bpp) for gw, gh, _ in geo[1:]]
            with stage_mb(1):
                counts = node.run_device_batch(d_in.data_ptr(), 0, nb,
                                               [0] + [o.data_ptr() for o in outs[1:]], s,
                                               stage_all=staged)
            torch.cuda.synchronize()
            for L in got:
                gw, gh, _ = geo[L]
                raw = outs[L][:counts[L] * gw * gh * bpp].cpu().numpy()
                got[L] += list(raw.view(dtype).reshape(counts[L], gh, gw))
            k0 += nb
    finally:
        node.close()
    ref = oracle.OracleDownsampler(geo, dtype, method)
    want = {L: [] for L in got}
    for f in frames:
        ref.add_frame(f)
        for L in want:
            r = ref.take_frame(L)
            if r is not None:
                want[L].append(r)
    for L in got:
        assert len(got[L]) == len(want[L]), (i, dims, devices, L)
        for k, (a, b) in enumerate(zip(got[L], want[L])):
            assert_parity(a, b, f"nodedev {i} {dims} L{L} frame {k}")


def test_node_device_batch_rejects(aqz):
    dims = [(TIME, 0, 1, 1), (SPACE, 16, 4, 1), (SPACE, 64, 32, 1), (SPACE, 64, 32, 1)]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    node = aqz.Node(geo, np.uint16, aqz.MEAN, [0, 0])
    try:
        assert node.unit == 4
        d_in = empty_device(6 * 64 * 64 * 2)
        bufs = [empty_device(6 * w * h * 2) for w, h, _ in geo[1:]]
        outs = [0] + [b.data_ptr() for b in bufs]
        with pytest.raises(aqz.AqzError) as e:
            node.run_device_batch(d_in.data_ptr(), 0, 6, outs)
        assert "shard units of 4" in str(e.value)
        with pytest.raises(aqz.AqzError) as e:
            node.run_device_batch(d_in.data_ptr(), 4096, 4, outs)
        assert "no HIP device" in str(e.value)
    finally:
        node.close()


@pytest.mark.parametrize("devices", [[0, 0], [1, 0], [0, 1]], ids=["0,0", "1,0", "0,1"])
def test_node_calls_leave_the_current_device(aqz, oracle, devices):
    """Every node entry point restores the caller thread's current HIP device
    (ADVICE r4): create, the stream calls, both batches and destroy, with the
    caller on device 0 and handles on other devices where the box has them."""
    torch = torch_cuda()
    if max(devices) >= torch.cuda.device_count():
        pytest.skip(f"needs {max(devices) + 1} GPUs")
    torch.cuda.set_device(0)
    geo = [(256, 128, 1), (128, 64, 1), (64, 32, 1)]
    rng = np.random.default_rng(4)
    frames = random_frames(rng, np.uint16, (4, 128, 256))

    def here():
        assert torch.cuda.current_device() == 0
    node = aqz.Node(geo, np.uint16, aqz.MEAN, devices)
    here()
    try:
        for f in frames[:2]:
            node.add_frame(f)
            here()
            node.take_frame(1)
            here()
        node.flush()
        here()
        outs = [None] + [np.empty(2 * w * h * 2, np.uint8) for w, h, _ in geo[1:]]
        node.run_host_batch(frames[2:].ctypes.data, 2, [0] + [o.ctypes.data for o in outs[1:]])
        here()
        d_in = to_device(frames)
        d_outs = [None] + [empty_device(4 * w * h * 2) for w, h, _ in geo[1:]]
        s = launch_stream()
        counts = node.run_device_batch(d_in.data_ptr(), 0, 4,
                                       [0] + [o.data_ptr() for o in d_outs[1:]], s)
        here()
        torch.cuda.synchronize()
        assert counts == [4, 4, 4]
        want = oracle.cascade_2d(frames[3], 3, aqz.MEAN)
        got = d_outs[2][3 * 64 * 32 * 2:].cpu().numpy().view(np.uint16).reshape(32, 64)
        assert np.array_equal(got, want[1])
    finally:
        node.close()
    here()


def test_node_device_batch_staging_grows_between_calls(aqz, oracle):
    """Staged blocks first in 1-unit sub-batches, then in one sub-batch of a
    larger budget (the staging grows: its streams drain first), then small
    again (the slots are reused as they are): three batches in a row equal
    one oracle stream."""
    torch = torch_cuda()
    geo = [(384, 200, 1), (192, 100, 1), (96, 50, 1), (48, 25, 1)]
    rng = np.random.default_rng(21)
    sizes = [5, 9, 4]
    frames = random_frames(rng, np.float32, (sum(sizes), 200, 384))
    node = aqz.Node(geo, np.float32, aqz.MEAN, [0, 0, 0])
    got = {L: [] for L in range(1, len(geo))}
    try:
        s = launch_stream()
        k0 = 0
        for nb, mb in zip(sizes, (1, 64, 1)):
            d_in = to_device(frames[k0:k0 + nb])
            outs = [None] + [empty_device(nb * w * h * 4) for w, h, _ in geo[1:]]
            with stage_mb(mb):
                c = node.run_device_batch(d_in.data_ptr(), 0, nb,
                                          [0] + [o.data_ptr() for o in outs[1:]], s,
                                          stage_all=True)
            torch.cuda.synchronize()
            assert c == [nb] * len(geo)
            for L in got:
                w, h, _ = geo[L]
                got[L] += list(outs[L].cpu().numpy().view(np.float32).reshape(nb, h, w))
            k0 += nb
    finally:
        node.close()
    ref = oracle.OracleDownsampler(geo, np.float32, aqz.MEAN)
    for k, f in enumerate(frames):
        ref.add_frame(f)
        for L in got:
            assert_parity(got[L][k], ref.take_frame(L), f"frame {k} L{L}")
