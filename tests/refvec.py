"""Vectors made by the REFERENCE ITSELF, and their replay.

tests/golden/make_reference_vectors.py runs acquire-zarr v0.8.1's own
zarr::Downsampler (oracle/_ref, compiled unmodified from
/root/reference/src/streaming/downsampler.cpp) over seeded inputs and stores
what it returned:

* tests/golden/reference_vectors.npz — per geometry x dtype the input
  frames (`in/<geom>/<dtype>`), and per case the take events
  (`ev/<case>`: rows of frame index, level, has_frame, nbytes) with the taken
  bytes concatenated in event order (`out/<case>`);
* tests/golden/reference_vectors.json — the manifest: each geometry's
  dimensions, frame count and take pattern, the reference's
  writer_configurations() per level (sizes, chunks, shards, scales), each
  method's downsampling_method() and get_metadata().dump(), and the messages
  the reference throws for an invalid dtype or method;
* tests/golden/reference_digests.json — per-level SHA-256 of every BASELINE
  config x method on tests/digest_util.py's splitmix64 inputs.

`replay(make_ds, ...)` feeds a case to any implementation offering
add_frame(np.ndarray) / take_frame(level) -> np.ndarray | None (the oracle on
the CPU, the HIP path on the GPU) and asserts byte equality with the
reference, frame readiness included.
"""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NPZ = os.path.join(GOLDEN, "reference_vectors.npz")
MANIFEST = os.path.join(GOLDEN, "reference_vectors.json")
DIGESTS = os.path.join(GOLDEN, "reference_digests.json")
NAN_NPZ = os.path.join(GOLDEN, "reference_nan_vectors.npz")

NP_DTYPES = [np.uint8, np.uint16, np.uint32, np.uint64, np.int8, np.int16,
             np.int32, np.int64, np.float32, np.float64]
METHOD_NAMES = ["decimate", "mean", "min", "max"]
SPACE, CHANNEL, TIME = 0, 1, 2

# name: (dims in storage order (type, size, chunk, shard), frames, take pattern)
#   take "all": every level after every frame (MultiscaleArray's loop,
#   multiscale.array.cpp:298-320); "every3": only after frames 2, 5, 8, ...,
#   so untaken frames meet the emplace rule (downsampler.cpp:599-605).
GEOMETRIES = {
    # odd XY at every level (edge replication), 3 levels
    "xy_odd_37x29": ([(TIME, 0, 2, 1), (SPACE, 37, 8, 1), (SPACE, 29, 8, 1)], 4, "all"),
    # even XY, 4 levels
    "xy_even_64x48": ([(TIME, 0, 1, 1), (SPACE, 64, 8, 1), (SPACE, 48, 8, 1)], 3, "all"),
    # XY halves twice, then levels that only copy (min(H,W) <= max chunk)
    "xy_copy_45x130": ([(TIME, 0, 1, 1), (SPACE, 45, 4, 1), (SPACE, 130, 16, 1)], 2, "all"),
    # untaken frames
    "xy_skip_33x17": ([(TIME, 0, 1, 1), (SPACE, 33, 8, 1), (SPACE, 17, 4, 1)], 7, "every3"),
    # odd Z = 15: the last plane passes through, two timepoints
    "z15_13x11": ([(TIME, 0, 1, 1), (SPACE, 15, 4, 1), (SPACE, 13, 4, 1), (SPACE, 11, 4, 1)],
                  30, "all"),
    # odd Z = 7 with odd XY
    "z7_9x7": ([(TIME, 0, 1, 1), (SPACE, 7, 2, 1), (SPACE, 9, 2, 1), (SPACE, 7, 2, 1)],
               14, "all"),
    # channels outside Z = 5, untaken frames
    "c2_z5_10x12": ([(TIME, 0, 1, 1), (CHANNEL, 2, 1, 1), (SPACE, 5, 2, 1), (SPACE, 10, 4, 1),
                     (SPACE, 12, 4, 1)], 20, "every3"),
    # Z halves while XY is copied
    "zonly_16_6x6": ([(TIME, 0, 1, 1), (SPACE, 16, 2, 1), (SPACE, 6, 8, 1), (SPACE, 6, 8, 1)],
                     16, "all"),
    # BASELINE config C1a, the reference's own example
    # (examples/stream-raw-multiscale-to-filesystem.c:13-67,80-90): 5-D
    # t10/5/2 c8/4/2 z6/2/1 y48/16/1 x64/16/2, frames i*1000+j (u16 wraps),
    # the 10 frames the example appends ...
    "example_5d": ([(TIME, 10, 5, 2), (CHANNEL, 8, 4, 2), (SPACE, 6, 2, 1), (SPACE, 48, 16, 1),
                    (SPACE, 64, 16, 2)], 10, "all"),
    # ... and one whole timepoint of that array (8 channels x 6 planes), so
    # every channel's Z pairs and the channel boundaries are pinned too
    "example_5d_t0": ([(TIME, 10, 5, 2), (CHANNEL, 8, 4, 2), (SPACE, 6, 2, 1), (SPACE, 48, 16, 1),
                       (SPACE, 64, 16, 2)], 48, "all"),
}

# geometries whose frames are the example's pattern, not seeded noise
EXAMPLE_GEOMETRIES = ("example_5d", "example_5d_t0")


def case_name(geom, dtype, method):
    return f"{geom}/{np.dtype(dtype).name}/{METHOD_NAMES[method]}"


def take_now(pattern, k):
    return pattern == "all" or (pattern == "every3" and k % 3 == 2)


def make_inputs(geom, dtype, seed):
    """Seeded frames for one geometry: full-range integers with blocks of the
    extremes (so 32/64-bit sums wrap and narrow ones truncate), or floats
    with NaN, +-inf, -0.0, subnormals, the largest finite values (sums that
    overflow) and large/small pairs (operation order)."""
    dims, n_frames, _ = GEOMETRIES[geom]
    h, w = dims[-2][1], dims[-1][1]
    dt = np.dtype(dtype)
    if geom in EXAMPLE_GEOMETRIES:
        # the example's `frame[j] = i * 1000 + j` into a uint16_t (mod 2^16),
        # the same numbers in every dtype
        i = np.arange(n_frames, dtype=np.int64)[:, None]
        j = np.arange(h * w, dtype=np.int64)[None, :]
        return ((i * 1000 + j) & 0xFFFF).astype(dt).reshape(n_frames, h, w)
    rng = np.random.default_rng(seed)
    shape = (n_frames, h, w)
    if dt.kind == "f":
        x = (rng.standard_normal(shape) * 1e3).astype(dt)
        fi = np.finfo(dt)
        specials = np.array([np.nan, np.inf, -np.inf, -0.0, 0.0, fi.max, -fi.max,
                             fi.smallest_subnormal, -fi.smallest_subnormal,
                             fi.smallest_subnormal * 3, fi.tiny, 1e8, -1e8, 1.0], dtype=dt)
        flat = x.reshape(-1)
        pos = rng.choice(flat.size, size=flat.size // 3, replace=False)
        flat[pos] = specials[rng.integers(0, specials.size, pos.size)]
        # whole 2x2 blocks of the largest value: the sum overflows to inf
        x[:, :2, :2] = fi.max
    else:
        ii = np.iinfo(dt)
        x = rng.integers(ii.min, ii.max, shape, dtype=dt, endpoint=True)
        flat = x.reshape(-1)
        ext = np.array([ii.min, ii.max, ii.min + 1, ii.max - 1, 0, -1 if ii.min < 0 else 1],
                       dtype=dt)
        pos = rng.choice(flat.size, size=flat.size // 3, replace=False)
        flat[pos] = ext[rng.integers(0, ext.size, pos.size)]
        x[:, :2, :2] = ii.max        # 4*max wraps in 32/64-bit arithmetic
        x[:, :2, 2:4] = ii.min
    return x


# NaN-payload cases (reference_nan_vectors.npz): the float dtypes over
# geometries that exercise mean4 with replicated edge operands (odd XY) and
# mean2 (Z pairs), on inputs dense in NaNs of every sign, payload and
# quietness, so the reference binary's NaN choice (first NaN operand,
# quieted; the negative default NaN for inf - inf) is pinned byte for byte.
NAN_GEOMETRIES = ["xy_odd_37x29", "z7_9x7", "c2_z5_10x12"]
NAN_DTYPES = [np.float32, np.float64]


def make_nan_inputs(geom, dtype, seed):
    """Frames whose elements are, in about equal parts, quiet NaNs, signaling
    NaNs (random sign and nonzero payload), +inf, -inf and ordinary values.
    Built on the bit patterns, so nothing on the way quiets a NaN."""
    dims, n_frames, _ = GEOMETRIES[geom]
    h, w = dims[-2][1], dims[-1][1]
    dt = np.dtype(dtype)
    ut = np.dtype(f"u{dt.itemsize}")
    nbits = 8 * dt.itemsize
    mant = 23 if dt.itemsize == 4 else 52
    rng = np.random.default_rng(seed)
    shape = (n_frames, h, w)
    x = (rng.standard_normal(shape) * 1e3).astype(dt)
    bits = x.view(ut).reshape(-1)
    kind = rng.integers(0, 5, bits.size)
    exp = ut.type(((1 << (nbits - 1 - mant)) - 1) << mant)
    sign = rng.integers(0, 2, bits.size).astype(ut) << ut.type(nbits - 1)
    quiet = ut.type(1 << (mant - 1))
    payload = rng.integers(1, 1 << (mant - 1), bits.size, dtype=np.uint64).astype(ut)
    qnan = sign | exp | quiet | (payload & ut.type(0xFF if mant == 23 else 0xFFFF))
    snan = sign | exp | payload               # quiet bit clear, payload nonzero
    inf = np.array(np.inf, dt).view(ut)
    ninf = np.array(-np.inf, dt).view(ut)
    bits[kind == 0] = qnan[kind == 0]
    bits[kind == 1] = snan[kind == 1]
    bits[kind == 2] = inf
    bits[kind == 3] = ninf
    return bits.view(dt).reshape(shape)


def nan_cases():
    return [(g, np.dtype(d).name, m) for g in NAN_GEOMETRIES for d in NAN_DTYPES
            for m in range(len(METHOD_NAMES))]


def load():
    with open(MANIFEST) as f:
        man = json.load(f)
    return man, np.load(NPZ, allow_pickle=False)


def cases(man):
    return [(g, d, m) for g in man["geometries"] for d in man["dtypes"]
            for m in range(len(METHOD_NAMES))]


def same(got_bytes, want_bytes, dt, nan_bits):
    """Byte equality; for floats with nan_bits=False, NaN positions must agree
    and every other value must be bit-identical (NaN payloads are not
    compared: x86 makes the negative default NaN for inf-inf, gfx950 the
    positive one; north_star's float bound is 1 ulp, and the rest is exact)."""
    if np.array_equal(got_bytes, want_bytes):
        return None
    if dt.kind != "f" or nan_bits:
        return np.flatnonzero(got_bytes != want_bytes)
    g, w = got_bytes.view(dt), want_bytes.view(dt)
    gn, wn = np.isnan(g), np.isnan(w)
    bad = np.flatnonzero((gn != wn) | (~gn & (g.view(f"u{dt.itemsize}") !=
                                              w.view(f"u{dt.itemsize}"))))
    return bad if bad.size else None


def replay(make_ds, man, vec, geom, dtype_name, method, nan_bits=True):
    """Feed the reference's inputs to `make_ds(dims, dtype, method)` and compare
    every take with the reference's events, byte for byte (see `same`)."""
    g = man["geometries"][geom]
    dt = np.dtype(dtype_name)
    frames = vec[f"in/{geom}/{dtype_name}"]
    name = f"{geom}/{dtype_name}/{METHOD_NAMES[method]}"
    ev = vec[f"ev/{name}"]
    out = vec[f"out/{name}"]
    ds = make_ds([tuple(d) for d in g["dims"]], dt, method)
    n_levels = len(g["levels"])
    i, off = 0, 0
    for k in range(frames.shape[0]):
        ds.add_frame(frames[k])
        if not take_now(g["take"], k):
            continue
        for L in range(1, n_levels):
            fk, fl, has, nb = (int(v) for v in ev[i])
            assert (fk, fl) == (k, L), f"{name}: event order {fk, fl} vs {k, L}"
            got = ds.take_frame(L)
            ctx = f"{name}: frame {k} level {L}"
            assert (got is not None) == bool(has), f"{ctx}: has_frame {got is not None}"
            if has:
                want = out[off:off + nb]
                b = np.ascontiguousarray(got).view(np.uint8).reshape(-1)
                assert b.size == nb, f"{ctx}: {b.size} bytes vs {nb}"
                bad = same(b, want, dt, nan_bits)
                if bad is not None:
                    raise AssertionError(f"{ctx}: {bad.size} elements differ, first at {bad[0]}")
                off += nb
            i += 1
    assert i == ev.shape[0] and off == out.size, name
