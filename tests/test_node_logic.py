"""CPU: the shard unit of aqz_node (frame sharding over a node's GPUs,
SURVEY §8(e)) — host logic only, no device call.

The property that makes sharding exact: feeding a stream through ONE
Downsampler, or cutting it into blocks of whole shard units and feeding each
block to a FRESH Downsampler, emits the same frames at every level in the
same order.  Checked with the oracle (whose state machine the reference
vectors pin, tests/test_reference_pin.py) on 2-D pyramids, even and odd Z
stacks, Z-only levels and channels outside Z; the emitted-per-unit counts
aqz_shard_unit reports must match what the blocks emitted."""
import numpy as np
import pytest

SPACE, CHANNEL, TIME = 0, 1, 2

GEOMS = {
    "2d": [(TIME, 0, 1, 1), (SPACE, 40, 8, 1), (SPACE, 36, 8, 1)],
    "z16": [(TIME, 0, 1, 1), (SPACE, 16, 4, 1), (SPACE, 20, 4, 1), (SPACE, 18, 4, 1)],
    "z12_odd_deep": [(TIME, 0, 1, 1), (SPACE, 12, 1, 1), (SPACE, 16, 8, 1), (SPACE, 16, 8, 1)],
    "z15": [(TIME, 0, 1, 1), (SPACE, 15, 4, 1), (SPACE, 13, 4, 1), (SPACE, 11, 4, 1)],
    "z7": [(TIME, 0, 1, 1), (SPACE, 7, 2, 1), (SPACE, 9, 2, 1), (SPACE, 7, 2, 1)],
    "zonly": [(TIME, 0, 1, 1), (SPACE, 16, 2, 1), (SPACE, 6, 8, 1), (SPACE, 6, 8, 1)],
    "c2_z5": [(TIME, 0, 1, 1), (CHANNEL, 2, 1, 1), (SPACE, 5, 2, 1), (SPACE, 10, 4, 1),
              (SPACE, 12, 4, 1)],
    "v256": [(TIME, 0, 1, 1), (SPACE, 256, 64, 1), (SPACE, 32, 8, 1), (SPACE, 32, 8, 1)],
}
EXPECT_UNIT = {"2d": 1, "z16": 4, "z12_odd_deep": 12, "z15": 15, "z7": 7, "zonly": 8,
               "c2_z5": 5, "v256": 4}


def _emitted(oracle, geo, frames, method):
    o = oracle.OracleDownsampler(geo, frames.dtype, method)
    out = {L: [] for L in range(1, len(geo))}
    for f in frames:
        o.add_frame(f)
        for L in out:
            r = o.take_frame(L)
            if r is not None:
                out[L].append(r)
    return out


@pytest.mark.parametrize("name", list(GEOMS))
def test_blocks_of_units_equal_one_stream(aqz, oracle, name):
    geo = aqz.level_geometry(aqz.plan_levels(GEOMS[name]))
    unit, per_unit = aqz.shard_unit(geo)
    assert unit == EXPECT_UNIT[name], (name, unit, geo)
    rng = np.random.default_rng(len(name))
    n_units = 5
    w, h, _ = geo[0]
    frames = rng.integers(0, 60000, (n_units * unit, h, w)).astype(np.uint16)
    for method in (1, 3):
        whole = _emitted(oracle, geo, frames, method)
        # ragged blocks of whole units, as a node deals them over 3 handles
        cuts = [0, 1, 3, 5]
        blocks = {L: [] for L in whole}
        for a, b in zip(cuts, cuts[1:]):
            part = _emitted(oracle, geo, frames[a * unit:b * unit], method)
            for L in blocks:
                assert len(part[L]) == (b - a) * per_unit[L], (name, L)
                blocks[L] += part[L]
        for L in whole:
            assert len(whole[L]) == n_units * per_unit[L]
            for x, y in zip(whole[L], blocks[L]):
                assert np.array_equal(x, y), (name, method, L)


def test_shard_unit_rejects_bad_levels(aqz):
    with pytest.raises(aqz.AqzError):
        aqz.shard_unit([])


def test_node_create_validates_before_any_device_call(aqz):
    import ctypes
    L = aqz.lib()
    geo = (aqz.LevelDesc * 2)(aqz.LevelDesc(10, 10, 1), aqz.LevelDesc(5, 5, 1))
    devs = (ctypes.c_int * 2)(0, 0)
    h = ctypes.c_void_p()
    assert L.aqz_node_create(geo, 2, 10, 1, devs, 2, ctypes.byref(h)) == 1
    assert "Invalid data type: 10" in L.aqz_last_error().decode()
    assert L.aqz_node_create(geo, 2, 1, 4, devs, 2, ctypes.byref(h)) == 1
    assert "Invalid downsampling method: 4" in L.aqz_last_error().decode()
    assert L.aqz_node_create(geo, 2, 1, 1, devs, 0, ctypes.byref(h)) == 1
    assert not h.value
