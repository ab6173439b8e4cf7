"""CPU: chunk-lattice addressing and multiscale level expectations pinned to
the reference's own tests (tests/golden/reference_kats.json).

* `addressing` — the 203 EXPECT_EQ assertions of
  tests/unit-tests/array-dimensions-{chunk-internal-offset,tile-group-offset,
  chunk-lattice-index}.cpp (t 0/5, c 3/2, z 5/2, y 48/16, x 64/16), which pin
  ArrayDimensions::chunk_lattice_index / tile_group_offset /
  chunk_internal_offset (array.dimensions.cpp:232-314).  Checked twice: the
  oracle's restatement (oracle/ds_oracle.c), and the product's
  aqz_chunk_frame_offsets through the C-ABI, whose offset of frame k is
  layer(k)·layer_bytes + tile_group_offset(k)·bytes_per_chunk +
  chunk_internal_offset(k) — decomposed back into the three reference
  quantities here.
* `integration` — per-level shapes, chunk and shard sizes and OME scales the
  multiscale integration tests expect (tests/integration/stream-3d-multiscale-
  to-filesystem.cpp, stream-multiscale-trivial-3rd-dim.cpp,
  stream-2d-multiscale-to-filesystem.cpp), against aqz_plan_levels (product)
  and oracle_plan_levels, plus the number of frames each level receives when
  the test's frames stream through the oracle state machine.
"""
import numpy as np
import pytest

import kat_runner

KATS = kat_runner.load()
ADDR = {c["function"]: c for c in KATS["addressing"]}
NP_DTYPES = kat_runner.NP_DTYPES


def _bpp(case):
    return np.dtype(NP_DTYPES[case["dtype"]]).itemsize


def test_fixture_holds_all_203_assertions():
    assert sum(len(c["asserts"]) for c in KATS["addressing"]) == 203
    assert set(ADDR) == {"chunk_internal_offset", "tile_group_offset", "chunk_lattice_index"}
    for c in KATS["addressing"]:
        assert c["dims"] == [[2, 0, 5, 0], [1, 3, 2, 0], [0, 5, 2, 0], [0, 48, 16, 0],
                             [0, 64, 16, 0]]


@pytest.mark.parametrize("fn", sorted(ADDR))
def test_oracle_reproduces_addressing_kats(oracle, fn):
    case = ADDR[fn]
    dims = case["dims"]
    for a in case["asserts"]:
        if fn == "chunk_internal_offset":
            got = oracle.chunk_internal_offset(dims, _bpp(case), a["args"][0])
        elif fn == "tile_group_offset":
            got = oracle.tile_group_offset(dims, a["args"][0])
        else:
            got = oracle.chunk_lattice_index(dims, *a["args"])
        assert got == a["expect"], f"line {a['line']}: {fn}{tuple(a['args'])} = {got}"


def _decompose(aqz, case, n_frames):
    """(layer, tile_group_offset, chunk_internal_offset) per frame 0..n-1 from
    the product's aqz_chunk_frame_offsets."""
    offs, cb, lb = aqz.chunk_frame_offsets(case["dims"], _bpp(case), 0, n_frames)
    return [(o // lb, (o % lb) // cb, o % cb) for o in offs], cb, lb


@pytest.mark.parametrize("fn", sorted(ADDR))
def test_product_offsets_reproduce_addressing_kats(aqz, fn):
    case = ADDR[fn]
    dims = case["dims"]
    n = max(a["args"][0] for a in case["asserts"]) + 1
    parts, cb, lb = _decompose(aqz, case, n)
    # bytes_per_chunk_ and one chunk layer (array.dimensions.cpp:168-178)
    assert cb == _bpp(case) * 5 * 2 * 2 * 16 * 16
    assert lb == 2 * 3 * 3 * 4 * cb
    # chunk-count strides of dims 1..2 inside a layer (tile_group_offset's)
    counts = [-(-d[1] // d[2]) for d in dims]
    stride = {1: counts[2] * counts[3] * counts[4], 2: counts[3] * counts[4]}
    for a in case["asserts"]:
        layer, tgo, cio = parts[a["args"][0]]
        if fn == "chunk_internal_offset":
            got = cio
        elif fn == "tile_group_offset":
            got = tgo
        else:
            d = a["args"][1]
            got = layer if d == 0 else (tgo // stride[d]) % counts[d]
        assert got == a["expect"], f"line {a['line']}: {fn}{tuple(a['args'])} = {got}"


def test_product_offsets_equal_oracle_addressing(aqz, oracle):
    """Beyond the KAT dims: random N-D dimension sets and batches starting
    mid-layer, the product's offsets against the oracle's literal
    restatement of the reference's stride loops."""
    rng = np.random.default_rng(11)
    for _ in range(200):
        nd = int(rng.integers(3, 7))
        dims = [(2, 0, int(rng.integers(1, 6)), 1)]
        for _ in range(nd - 3):
            size = int(rng.integers(1, 8))
            dims.append((1, size, int(rng.integers(1, size + 1)), 1))
        for _ in range(2):
            size = int(rng.integers(1, 400))
            dims.append((0, size, int(rng.integers(1, 100)), 1))
        bpp = int(rng.choice([1, 2, 4, 8]))
        first = int(rng.integers(0, 300))
        got = aqz.chunk_frame_offsets(dims, bpp, first, 30)
        want = oracle.chunk_frame_offsets(dims, bpp, first, 30)
        assert got == want, dims


INTEG = {c["name"]: c for c in KATS["integration"]}


def _dims(case):
    return [tuple(d) for d in case["dims"]]


def _check_scale(got, want, rule, ctx):
    if rule == "int":
        # the reference compares through EXPECT_EQ(int, ...): truncated
        assert int(got) == int(want), ctx
    # and the planner's scale is the exact product (scale *= 2 per halving,
    # downsampler.cpp:8-37), which is what the metadata carries
    assert got == pytest.approx(want, rel=0, abs=1e-12), ctx


@pytest.mark.parametrize("planner", ["product", "oracle"])
@pytest.mark.parametrize("name", ["stream_3d_multiscale", "stream_2d_multiscale"])
def test_integration_level_geometry(aqz, oracle, planner, name):
    case = INTEG[name]
    plan = aqz.plan_levels if planner == "product" else oracle.plan_levels
    levels = plan(_dims(case))
    assert len(levels) == case["n_levels"]
    for L, want in enumerate(case["levels"]):
        lv = levels[L]
        ctx = f"{name} L{L}"
        sizes = [d[1] for d in lv]
        # the append dimension keeps its configured size at every level
        assert sizes == want["sizes"], ctx
        assert [d[2] for d in lv] == want["chunks"], ctx
        assert [d[3] for d in lv] == want["shards"], ctx
        for i, (d, s) in enumerate(zip(lv, want["scales"])):
            _check_scale(d[4], s, case["scale_rule"], f"{ctx} dim {i}")


@pytest.mark.parametrize("planner", ["product", "oracle"])
def test_trivial_third_dim_levels(aqz, oracle, planner):
    """stream-multiscale-trivial-3rd-dim.cpp: z = 1 is never downsampled
    (scale stays 1.36), t/c scales stay 1.0, y/x scales are 0.85 x (base size
    / level size, integer division) within 0.01, 3 datasets."""
    case = INTEG["stream_multiscale_trivial_3rd_dim"]
    plan = aqz.plan_levels if planner == "product" else oracle.plan_levels
    levels = plan(_dims(case))
    assert len(levels) == case["n_levels"]
    rel = case["scale_relation"]
    base = levels[0]
    for L, lv in enumerate(levels):
        for i in rel["fixed"]:
            assert lv[i][1] == base[i][1] and lv[i][4] == rel["base_scale"][i], (L, i)
        for i in rel["ratio"]:
            want = rel["base_scale"][i] * (base[i][1] // lv[i][1])
            assert abs(lv[i][4] - want) < 0.01, (L, i, lv[i][4], want)
        if L:
            assert lv[3][1] < levels[L - 1][3][1] and lv[4][1] < levels[L - 1][4][1]


def _stream_counts(oracle, case, geo, n_frames, zero):
    dtype = NP_DTYPES[case["dtype"]]
    ds = oracle.OracleDownsampler(geo, dtype, case["method"])
    rng = np.random.default_rng(5)
    counts = [0] * len(geo)
    w, h, _ = geo[0]
    for _ in range(n_frames):
        fr = np.zeros((h, w), dtype) if zero else rng.integers(0, 65535, (h, w)).astype(dtype)
        ds.add_frame(fr)
        counts[0] += 1
        for L in range(1, len(geo)):
            if ds.take_frame(L) is not None:
                counts[L] += 1
    return counts


@pytest.mark.parametrize("name", ["stream_3d_multiscale", "stream_2d_multiscale"])
def test_integration_frames_per_level(aqz, oracle, name):
    """Frames each level's array receives (the shapes' append extents follow
    from them, stream-3d...cpp:240-255): all 480 frames of the 3-D test give
    240 at level 1 and 160 at level 2; the 2-D test's 80 reach every level."""
    case = INTEG[name]
    geo = aqz.level_geometry(aqz.plan_levels(_dims(case)))
    counts = _stream_counts(oracle, case, geo, case["levels"][0]["frames"], False)
    assert counts == [lv["frames"] for lv in case["levels"]]
