"""Replays tests/golden/reference_kats.json against any implementation that
offers the Downsampler surface: add_frame(np.ndarray) / take_frame(level) ->
np.ndarray | None.  Used for the oracle (CPU) and the HIP path (GPU)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                      "reference_kats.json")
NP_DTYPES = [np.uint8, np.uint16, np.uint32, np.uint64, np.int8, np.int16,
             np.int32, np.int64, np.float32, np.float64]


def load():
    with open(GOLDEN) as f:
        return json.load(f)


def full_dims(case):
    """(type, size, chunk, shard, scale) tuples.  The reference's 2-D tests use
    3 dimensions (t, y, x), so no phantom dimension is involved."""
    return [tuple(d) + (1.0,) for d in case["dims"]]


def frame_of(spec, dtype):
    if spec["kind"] == "const":
        return np.full((spec["h"], spec["w"]), spec["value"], dtype=dtype)
    return np.array(spec["data"], dtype=dtype)


def check_take(got, want, ctx):
    if want is None:
        assert got is None, f"{ctx}: expected no frame"
        return
    assert got is not None, f"{ctx}: expected a frame"
    assert got.shape == (want["h"], want["w"]), f"{ctx}: shape {got.shape}"
    if "all" in want:
        assert np.all(got == want["all"]), f"{ctx}: values {np.unique(got)[:8]}"
    else:
        np.testing.assert_array_equal(got, np.array(want["data"], dtype=got.dtype),
                                      err_msg=ctx)


def run_stream_case(case, make_ds):
    """`make_ds(geometry, dtype, method)` builds the implementation under test;
    geometry is derived by `plan(dims)` inside make_ds's caller."""
    dtype = NP_DTYPES[case["dtype"]]
    ds = make_ds(case, dtype, case["method"])
    seq = []
    for i, step in enumerate(case["steps"]):
        ds.add_frame(frame_of(step["add"], dtype))
        if step.get("take_any"):
            got = ds.take_frame(1)
            if got is not None:
                assert np.all(got == got.flat[0])
                seq.append(int(got.flat[0]))
        for level, want in step.get("take", []):
            check_take(ds.take_frame(level), want, f"{case['name']} step {i} L{level}")
    if "level1_sequence" in case:
        assert seq == case["level1_sequence"], f"{case['name']}: {seq}"
        assert ds.take_frame(1) is None
