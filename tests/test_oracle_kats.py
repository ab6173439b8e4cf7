"""CPU: pin the oracle (oracle/ds_oracle.c) to the reference's own known
answers before it is trusted as the GPU parity checker.

* tests/golden/reference_kats.json — the KATs of the reference's unit tests
  (tests/unit-tests/downsampler.cpp, downsampler-odd-z.cpp) and the example
  geometry, as data;
* SURVEY.md §0 [probe] scalar facts about the reference arithmetic;
* python/tests/test_stream.py pixel expectations (scikit-image / numpy
  semantics restated in tests/published_semantics.py).
"""
import numpy as np
import pytest

import kat_runner
import published_semantics as ps

KATS = kat_runner.load()


def _oracle_ds(oracle):
    def make(case, dtype, method):
        levels = oracle.plan_levels(kat_runner.full_dims(case))
        return oracle.OracleDownsampler(oracle.level_geometry(levels), dtype, method)
    return make


@pytest.mark.parametrize("case", KATS["planner"], ids=lambda c: c["name"])
def test_planner_kats(oracle, case):
    levels = oracle.plan_levels(kat_runner.full_dims(case), case["max_levels"])
    if "n_levels" in case:
        assert len(levels) == case["n_levels"]
    if "n_levels_gt" in case:
        assert len(levels) > case["n_levels_gt"]
    for lv, sizes in enumerate(case.get("sizes", [])):
        assert [d[1] for d in levels[lv]] == sizes, f"level {lv}"
    for lv, chunks in enumerate(case.get("chunks", [])):
        assert [d[2] for d in levels[lv]] == chunks, f"level {lv}"
    if "level1_dim1_size" in case:
        assert levels[1][1][1] == case["level1_dim1_size"]


@pytest.mark.parametrize("case", KATS["stream"], ids=lambda c: c["name"])
def test_stream_kats(oracle, case):
    kat_runner.run_stream_case(case, _oracle_ds(oracle))


def test_survey_probe_scalars(oracle):
    """Facts probed on the reference binary."""
    # int8 mean truncates toward zero: (-1-2-3-1)/4 = -7/4 -> -1
    assert oracle.reduce4(np.int8, oracle.MEAN, -1, -2, -3, -1) == -1
    # uint32 sums wrap: 4*0xFFFFFFFF mod 2^32 = 0xFFFFFFFC, /4
    assert oracle.reduce4(np.uint32, oracle.MEAN, *[0xFFFFFFFF] * 4) == 1073741823
    # float sums run left to right: ((1e8 + 1) - 1e8) + 1 = 1 -> 0.25
    assert oracle.reduce4(np.float32, oracle.MEAN, 1e8, 1, -1e8, 1) == np.float32(0.25)
    # odd edges replicate: 3x3 u16 1..9 -> [[3, 4], [7, 9]]
    img = np.arange(1, 10, dtype=np.uint16).reshape(3, 3)
    np.testing.assert_array_equal(oracle.scale_image(img, oracle.MEAN),
                                  np.array([[3, 4], [7, 9]], dtype=np.uint16))


def test_compare_select_nan_order(oracle):
    """min/max are `b < val` chains seeded with the first operand
    (downsampler.cpp:64-98): NaN first -> NaN, NaN later -> skipped."""
    nan = np.float32(np.nan)
    assert np.isnan(oracle.reduce4(np.float32, oracle.MIN, nan, 1, 2, 3))
    assert oracle.reduce4(np.float32, oracle.MIN, 5, nan, 2, 3) == 2
    # max2 is `a > b ? a : b` (downsampler.cpp:133-137): a NaN `a` loses
    assert oracle.reduce2(np.float32, oracle.MAX, nan, 1) == 1
    assert np.isnan(oracle.reduce2(np.float32, oracle.MAX, 1, nan))
    # decimate keeps the earlier plane / top-left pixel
    assert oracle.reduce2(np.int16, oracle.DECIMATE, -5, 7) == -5


def _mean_bits(oracle, ut, bits):
    """The oracle's mean4 (4 operands) or mean2 (2) on raw bit patterns, so
    no float conversion on the way quiets a signaling NaN."""
    dt = np.float32 if ut is np.uint32 else np.float64
    v = np.array(bits, dtype=ut).view(dt)
    out = np.zeros(1, dtype=dt)
    p, isz = v.ctypes.data, v.itemsize
    code = oracle.dtype_code(dt)
    if len(bits) == 4:
        oracle.lib().oracle_reduce4(code, oracle.MEAN, p, p + isz, p + 2 * isz, p + 3 * isz,
                                    out.ctypes.data)
    else:
        oracle.lib().oracle_reduce2(code, oracle.MEAN, p, p + isz, out.ctypes.data)
    return int(out.view(ut)[0])


def test_mean_nan_payload_rule(oracle):
    """The reference binary's NaN result (x86 SSE addss/divss in the order
    ((a + b) + c) + d, downsampler.cpp:48-51,108-112), which the GPU restates
    (ds_kernels.hip x86_add): the first NaN operand wins, quieted; an invalid
    sum (inf + -inf) gives the negative default NaN; a quiet NaN survives
    the later adds and the divide.  Pinned against the reference itself by
    tests/golden/reference_nan_vectors.npz (test_reference_pin.py)."""
    inf, ninf, one = 0x7F800000, 0xFF800000, 0x3F800000
    qa, qb = 0x7FC01234, 0xFFC0ABCD          # quiet, payloads, both signs
    sa = 0x7F800F00                          # signaling (quiet bit clear)
    u = np.uint32
    assert _mean_bits(oracle, u, [qa, qb, one, one]) == qa          # first NaN
    assert _mean_bits(oracle, u, [one, qb, qa, one]) == qb
    assert _mean_bits(oracle, u, [sa, one, one, one]) == sa | 0x00400000  # quieted
    assert _mean_bits(oracle, u, [one, sa, qa, one]) == sa | 0x00400000
    assert _mean_bits(oracle, u, [inf, ninf, one, one]) == 0xFFC00000   # default NaN
    assert _mean_bits(oracle, u, [inf, ninf, qa, one]) == 0xFFC00000   # made first
    assert _mean_bits(oracle, u, [one, inf, one, ninf]) == 0xFFC00000
    assert _mean_bits(oracle, u, [qb, inf, ninf, one]) == qb
    assert _mean_bits(oracle, u, [qa, qb]) == qa                        # mean2
    assert _mean_bits(oracle, u, [inf, ninf]) == 0xFFC00000
    d = np.uint64
    assert _mean_bits(oracle, d, [0x7FF0000000000001, 0x7FF8000000000002]) == \
        0x7FF8000000000001
    assert _mean_bits(oracle, d, [0x7FF0000000000000, 0xFFF0000000000000, 0, 0]) == \
        0xFFF8000000000000


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_2d_stream_expectations(oracle, method):
    """test_2d_multiscale_stream (test_stream.py:993-1077): int32 in
    [-2^16, 2^16-1), 48x64 frames, level 1 equals the scikit-image/numpy
    reduction cast to int32, exactly."""
    rng = np.random.default_rng(1234 + method)
    levels = oracle.plan_levels([(oracle.TIME, 50, 50, 1), (oracle.SPACE, 48, 24, 1),
                                 (oracle.SPACE, 64, 32, 1)])
    geo = oracle.level_geometry(levels)
    assert geo[1][:2] == (32, 24)
    ds = oracle.OracleDownsampler(geo, np.int32, method)
    ref = {0: ps.decimate, 1: ps.downscale_local_mean, 2: ps.block_reduce_min,
           3: ps.block_reduce_max}[method]
    for _ in range(50):
        x = rng.integers(-(2 ** 16), 2 ** 16 - 1, (48, 64), dtype=np.int32)
        ds.add_frame(x)
        got = ds.take_frame(1)
        np.testing.assert_array_equal(got, ref(x).astype(np.int32))


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_3d_stream_expectations(oracle, method):
    """test_3d_multiscale_stream (test_stream.py:1080-1190): z=100 u16,
    level 1 is 50 planes; Mean within atol=1 of the float reference, the other
    methods exact."""
    rng = np.random.default_rng(99 + method)
    levels = oracle.plan_levels([(oracle.SPACE, 100, 50, 1), (oracle.SPACE, 48, 24, 1),
                                 (oracle.SPACE, 64, 32, 1)])
    geo = oracle.level_geometry(levels)
    assert geo[1] == (32, 24, 50)
    ds = oracle.OracleDownsampler(geo, np.uint16, method)
    data = rng.integers(0, 2 ** 16 - 1, (100, 48, 64), dtype=np.uint16)
    out = []
    for z in range(100):
        ds.add_frame(data[z])
        f = ds.take_frame(1)
        if f is not None:
            out.append(f)
    assert len(out) == 50
    for i, actual in enumerate(out):
        a, b = data[2 * i], data[2 * i + 1]
        if method == 1:
            e = ((ps.downscale_local_mean(a) + ps.downscale_local_mean(b)) / 2).astype(np.uint16)
            np.testing.assert_allclose(e, actual, atol=1)
        elif method == 0:
            np.testing.assert_array_equal(actual, ps.decimate(a))
        elif method == 2:
            np.testing.assert_array_equal(actual, np.minimum(ps.block_reduce_min(a),
                                                             ps.block_reduce_min(b)))
        else:
            np.testing.assert_array_equal(actual, np.maximum(ps.block_reduce_max(a),
                                                             ps.block_reduce_max(b)))


def test_no_lod_bleed_expectation(oracle):
    """test_odd_z_multi_channel_no_lod_bleed (test_stream.py:1193-1271)."""
    T, C, Z, Y, X = 2, 2, 3, 8, 8
    levels = oracle.plan_levels([(oracle.TIME, T, 1, T), (oracle.CHANNEL, C, 1, C),
                                 (oracle.SPACE, Z, 1, Z), (oracle.SPACE, Y, Y, 1),
                                 (oracle.SPACE, X, X, 1)])
    geo = oracle.level_geometry(levels)
    assert geo[1][2] == (Z + 1) // 2
    ds = oracle.OracleDownsampler(geo, np.uint16, oracle.MEAN)
    lod1 = []
    for t in range(T):
        for c, v in enumerate((100, 200)):
            for z in range(Z):
                ds.add_frame(np.full((Y, X), v, np.uint16))
                f = ds.take_frame(1)
                if f is not None:
                    lod1.append((t, c, int(f.flat[0]), bool(np.all(f == f.flat[0]))))
    assert len(lod1) == T * C * ((Z + 1) // 2)
    for t, c, v, uniform in lod1:
        assert uniform and v == (100, 200)[c]


def test_emplace_does_not_overwrite(oracle):
    """emplace_downsampled_frame_ (downsampler.cpp:599-605) keeps the first
    untaken frame; the count still moves."""
    levels = oracle.plan_levels([(oracle.TIME, 0, 5, 1), (oracle.SPACE, 10, 5, 1),
                                 (oracle.SPACE, 10, 5, 1)])
    ds = oracle.OracleDownsampler(oracle.level_geometry(levels), np.uint8, oracle.MEAN)
    ds.add_frame(np.full((10, 10), 10, np.uint8))
    ds.add_frame(np.full((10, 10), 20, np.uint8))
    assert ds.level_count(1) == 2
    assert np.all(ds.take_frame(1) == 10)
    assert ds.take_frame(1) is None


def test_tile_frame_geometry_and_bytes(oracle):
    """Chunk tiling oracle: the reference's array tests use 64x48 frames in
    16x16 chunks -> 4x3 tiles (tests/unit-tests/array-write-even.cpp:26-29);
    ragged tiles are zero-padded in the chunk buffer; the nonzero flag is the
    chunk zero scan.  Checked against an independent numpy pad+reshape."""
    rng = np.random.default_rng(3)
    for (h, w, tr, tc, dt) in [(48, 64, 16, 16, np.uint16), (50, 70, 16, 32, np.float32),
                               (7, 300, 4, 128, np.uint8), (33, 33, 64, 64, np.int64)]:
        img = rng.integers(1, 100, (h, w)).astype(dt)
        img[:tr, :tc] = 0  # an all-zero first tile
        tiles, nz = oracle.tile_frame(img, tr, tc)
        nty, ntx = -(-h // tr), -(-w // tc)
        assert tiles.shape == (nty * ntx, tr, tc)
        pad = np.zeros((nty * tr, ntx * tc), dt)
        pad[:h, :w] = img
        want = pad.reshape(nty, tr, ntx, tc).transpose(0, 2, 1, 3).reshape(-1, tr, tc)
        np.testing.assert_array_equal(tiles, want)
        assert not nz[0] and nz[1:].all()


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.int32, np.float32,
                                   np.uint64, np.float64],
                         ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("shape", [(1, 1), (1, 7), (7, 1), (30, 20), (65, 129)])
def test_oracle_transpose_frame(oracle, dtype, shape):
    """transpose_frame restatement (array.cpp:488-504) against numpy's
    transpose, which is what python/tests/test_stream.py::
    test_write_transposed_array expects the stored array to equal
    (np.transpose(data, (0, 1, 2, 4, 3)) for a t,c,z,x,y acquisition)."""
    rng = np.random.default_rng(sum(shape))
    frame = rng.integers(0, 255, size=shape).astype(dtype)
    got = oracle.transpose_frame(frame)
    assert got.shape == shape[::-1]
    assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(frame.T).view(np.uint8))
