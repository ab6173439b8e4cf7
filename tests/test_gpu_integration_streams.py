"""GPU: the reference's multiscale integration tests' streams through the HIP
path (aqz::Downsampler over the C-ABI), against the oracle frame by frame.

Geometry and per-level frame counts come from tests/golden/reference_kats.json
(`integration`, transcribed from tests/integration/stream-3d-multiscale-to-
filesystem.cpp, stream-multiscale-trivial-3rd-dim.cpp and
stream-2d-multiscale-to-filesystem.cpp); the CPU suite pins the planner to
them (tests/test_reference_addressing.py).  The reference streams zeros; here
random frames are streamed too, so every level's pixels are checked as well
as its readiness.
"""
import numpy as np
import pytest

import kat_runner
from gpu_util import assert_parity

pytestmark = pytest.mark.gpu

INTEG = {c["name"]: c for c in kat_runner.load()["integration"]}


def _frames_in(case):
    return case["frames_in"] if "frames_in" in case else case["levels"][0]["frames"]


@pytest.mark.parametrize("zero", [True, False], ids=["zeros", "random"])
@pytest.mark.parametrize("name", sorted(INTEG))
@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_integration_stream(aqz, oracle, name, zero, method):
    case = INTEG[name]
    dims = [tuple(d) for d in case["dims"]]
    levels = aqz.plan_levels(dims)
    assert levels == oracle.plan_levels(dims)
    geo = aqz.level_geometry(levels)
    assert len(geo) == case["n_levels"]
    dtype = kat_runner.NP_DTYPES[case["dtype"]]
    ds = aqz.Downsampler(geo, dtype, method, device=0)
    ref = oracle.OracleDownsampler(geo, dtype, method)
    rng = np.random.default_rng(17 + method)
    w, h, _ = geo[0]
    counts = [0] * len(geo)
    for i in range(_frames_in(case)):
        fr = (np.zeros((h, w), dtype) if zero
              else rng.integers(0, 65536, (h, w)).astype(dtype))
        ds.add_frame(fr)
        ref.add_frame(fr)
        counts[0] += 1
        for L in range(1, len(geo)):
            a, b = ds.take_frame(L), ref.take_frame(L)
            assert (a is None) == (b is None), f"{name} frame {i} L{L}"
            if a is not None:
                counts[L] += 1
                assert_parity(a, b, f"{name} m{method} frame {i} L{L}")
                if zero:
                    assert not a.any()
    ds.close()
    if "levels" in case:
        assert counts == [lv["frames"] for lv in case["levels"]]
    else:
        # z = 1 is never halved: every frame reaches every level
        assert counts == [_frames_in(case)] * len(geo)
