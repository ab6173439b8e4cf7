"""CPU: the C-ABI library loads, exports every function include/*.h declares,
and its host-only entry points (planner, method strings) agree with the
oracle and the reference text.  No GPU compute is called here."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

import kat_runner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    names = set()
    inc = os.path.join(ROOT, "include")
    for h in sorted(os.listdir(inc)):
        if h.endswith(".h"):
            src = re.sub(r"/\*.*?\*/", "", open(os.path.join(inc, h)).read(), flags=re.S)
            names |= set(re.findall(r"\b(aqz_\w+)\s*\(", src))
    return sorted(names)


def test_library_exports_header(aqz):
    lib = aqz.lib()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), f"missing export {n}"
    assert set(names) == set(aqz.EXPORTS)


def test_library_is_gfx950(aqz):
    blob = open(aqz.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_method_strings(aqz):
    # Downsampler::downsampling_method (downsampler.cpp:422-437)
    assert [aqz.method_name(m) for m in range(4)] == [
        "decimate", "local_mean", "local_min", "local_max"]
    assert aqz.method_name(4) is None
    # Downsampler::get_metadata (downsampler.cpp:440-485)
    md = aqz.method_metadata(aqz.MEAN)
    assert md["method"] == "skimage.transform.downscale_local_mean"
    assert md["kwargs"] == {"factors": "(2, 2)", "cval": "0"}
    assert md["version"] == "0.25.2"
    assert aqz.method_metadata(aqz.DECIMATE)["args"] == [
        "(slice(0, None, 2), slice(0, None, 2))"]
    assert aqz.method_metadata(aqz.MIN)["kwargs"] == {"func": "np.min"}
    assert aqz.method_metadata(aqz.MAX)["kwargs"] == {"func": "np.max"}


KATS = kat_runner.load()


@pytest.mark.parametrize("case", KATS["planner"], ids=lambda c: c["name"])
def test_product_planner_kats(aqz, case):
    levels = aqz.plan_levels(kat_runner.full_dims(case), case["max_levels"])
    if "n_levels" in case:
        assert len(levels) == case["n_levels"]
    if "n_levels_gt" in case:
        assert len(levels) > case["n_levels_gt"]
    for lv, sizes in enumerate(case.get("sizes", [])):
        assert [d[1] for d in levels[lv]] == sizes
    for lv, chunks in enumerate(case.get("chunks", [])):
        assert [d[2] for d in levels[lv]] == chunks


def test_product_planner_matches_oracle(aqz, oracle):
    """Random dimension sets, including odd sizes, anisotropic chunks,
    non-spatial Z and max_levels caps."""
    rng = np.random.default_rng(7)
    for _ in range(2000):
        nd = int(rng.integers(3, 6))
        dims = []
        for i in range(nd):
            kind = int(rng.integers(0, 4)) if i < nd - 2 else 0
            size = int(rng.integers(1, 5000))
            chunk = int(rng.integers(1, 600))
            shard = int(rng.integers(1, 9))
            dims.append((kind, size, chunk, shard, float(rng.uniform(0.1, 3))))
        ml = int(rng.integers(0, 6))
        a = aqz.plan_levels(dims, ml)
        b = oracle.plan_levels(dims, ml)
        assert a == b, (dims, ml)


def test_planner_rejects_bad_dims(aqz):
    with pytest.raises(aqz.AqzError):
        aqz.plan_levels([(0, 10, 0, 1), (0, 10, 5, 1), (0, 10, 5, 1)])


def test_create_rejects_bad_arguments_without_gpu(aqz):
    """Argument validation happens before any device call."""
    geo = [(10, 10, 1), (5, 5, 1)]
    with pytest.raises(aqz.AqzError) as e:
        aqz.Downsampler(geo, np.uint8, 9)
    assert e.value.status == 1 and "method" in str(e.value)
    with pytest.raises(aqz.AqzError):
        aqz.Downsampler([(10, 10, 1), (4, 4, 1)], np.uint8, 1)
