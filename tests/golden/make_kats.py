"""Generate tests/golden/reference_kats.json.

The fixtures are the known-answer cases the reference's own test-suite holds
for the downsampler (acquire-zarr v0.8.1), written down as data: the level
configuration, the input frames and the expected outputs / level geometry /
frame-readiness sequence.  Every value comes from the cited reference test;
nothing here is computed by the oracle or the product.

Sources:
  R1 tests/unit-tests/downsampler.cpp
  R2 tests/unit-tests/downsampler-odd-z.cpp
  R3 examples/stream-raw-multiscale-to-filesystem.c (BASELINE config 0)

The reference cannot be compiled in this image (src/streaming/downsampler.hh
includes nlohmann/json.hpp, which is absent) and its Python package cannot be
built, so no fixture was produced by running reference code.

Run: python tests/golden/make_kats.py
"""
from __future__ import annotations

import json
import os

SPACE, CHANNEL, TIME, OTHER = 0, 1, 2, 3
DECIMATE, MEAN, MIN, MAX = 0, 1, 2, 3
U8, U16, U32, U64, I8, I16, I32, I64, F32, F64 = range(10)
ALL_DTYPES = [U8, U16, U32, U64, I8, I16, I32, I64, F32, F64]


def dim(t, size, chunk, shard=1):
    return [t, size, chunk, shard]


def const_frame(w, h, v):
    return {"kind": "const", "w": w, "h": h, "value": v}


def planner_cases():
    cases = []
    # R1 test_writer_configurations (:256-314): 5 levels; spatial sizes are
    # max(chunk, size / 2^level); t and c untouched.
    dims = [dim(TIME, 100, 10), dim(CHANNEL, 3, 3), dim(SPACE, 128, 8),
            dim(SPACE, 512, 64), dim(SPACE, 512, 64)]
    levels = []
    for lv in range(5):
        levels.append([100, 3] + [max(d[2], d[1] // (1 << lv)) for d in dims[2:]])
    cases.append({"name": "writer_configurations", "src": "R1:256-314",
                  "dims": dims, "max_levels": 0, "n_levels": 5,
                  "sizes": levels})
    # R1 test_anisotropic_writer_configurations (:316-409)
    dims = [dim(TIME, 100, 10), dim(CHANNEL, 3, 3), dim(SPACE, 1000, 128),
            dim(SPACE, 2000, 512), dim(SPACE, 2000, 256)]
    cases.append({"name": "anisotropic_writer_configurations", "src": "R1:316-409",
                  "dims": dims, "max_levels": 0, "n_levels": 4,
                  "sizes": [[100, 3, 1000, 2000, 2000], [100, 3, 500, 1000, 1000],
                            [100, 3, 250, 500, 500], [100, 3, 125, 500, 500]],
                  "chunks": [[10, 3, 128, 512, 256]] * 4})
    # R1 test_max_levels (:730-785): max_levels=2 -> 3 configurations; 0 -> >3
    dims = [dim(TIME, 100, 10), dim(SPACE, 512, 64), dim(SPACE, 512, 64)]
    cases.append({"name": "max_levels_2", "src": "R1:741-765", "dims": dims,
                  "max_levels": 2, "n_levels": 3, "two_d": True})
    cases.append({"name": "max_levels_none", "src": "R1:767-784", "dims": dims,
                  "max_levels": 0, "n_levels_gt": 3, "two_d": True})
    # R1 test_basic_downsampling (:29-50): 2 configurations
    cases.append({"name": "basic_2d_10x10", "src": "R1:29-50",
                  "dims": [dim(TIME, 0, 5), dim(SPACE, 10, 5), dim(SPACE, 10, 5)],
                  "max_levels": 0, "n_levels": 2, "two_d": True})
    # R2 main (:140-165): z=15 chunk 3 -> level-1 z = 8
    cases.append({"name": "odd_z_15", "src": "R2:140-165",
                  "dims": [dim(TIME, 0, 1), dim(SPACE, 15, 3), dim(SPACE, 48, 16),
                           dim(SPACE, 64, 16)],
                  "max_levels": 0, "level1_dim1_size": 8})
    # R3 example: t10 c8 z6/2 y48/16 x64/16 -> z/y/x 6/48/64, 3/24/32, 2/12/16
    # (level sizes derived in SURVEY.md §0 item 7 from the reference planner)
    cases.append({"name": "example_5d", "src": "R3:29-65",
                  "dims": [dim(TIME, 10, 5, 2), dim(CHANNEL, 8, 4, 2),
                           dim(SPACE, 6, 2, 1), dim(SPACE, 48, 16, 1),
                           dim(SPACE, 64, 16, 2)],
                  "max_levels": 0, "n_levels": 3,
                  "sizes": [[10, 8, 6, 48, 64], [10, 8, 3, 24, 32], [10, 8, 2, 12, 16]]})
    return cases


def stream_cases():
    """add_frame / take_frame sequences with expected results."""
    cases = []
    d2_10 = [dim(TIME, 0, 5), dim(SPACE, 10, 5), dim(SPACE, 10, 5)]
    # R1 test_basic_downsampling (:52-73)
    cases.append({"name": "basic_mean_u8", "src": "R1:52-73", "dims": d2_10,
                  "two_d": True, "dtype": U8, "method": MEAN,
                  "steps": [{"add": const_frame(10, 10, 100),
                             "take": [[1, {"w": 5, "h": 5, "all": 100}],
                                      [1, None]]}]})
    # R1 test_data_types (:154-254): every dtype gives a 5x5 level 1
    for dt in ALL_DTYPES:
        cases.append({"name": f"data_type_{dt}", "src": "R1:154-254",
                      "dims": d2_10, "two_d": True, "dtype": dt, "method": MEAN,
                      "steps": [{"add": const_frame(10, 10, 100),
                                 "take": [[1, {"w": 5, "h": 5, "all": 100}]]}]})
    # R1 test_edge_cases (:411-445): 11x11 -> 6x6
    cases.append({"name": "odd_11x11", "src": "R1:411-445",
                  "dims": [dim(TIME, 0, 5), dim(SPACE, 11, 5), dim(SPACE, 11, 5)],
                  "two_d": True, "dtype": U8, "method": MEAN,
                  "steps": [{"add": const_frame(11, 11, 100),
                             "take": [[1, {"w": 6, "h": 6, "all": 100}]]}]})
    # R1 test_min_max_downsampling (:447-528): blocks [100 200; 150 250]
    block = []
    for y in range(10):
        block.append([(100 if x % 2 == 0 else 200) if y % 2 == 0
                      else (150 if x % 2 == 0 else 250) for x in range(10)])
    for m, want in ((MEAN, 175), (MIN, 100), (MAX, 250)):
        cases.append({"name": f"blocks_method_{m}", "src": "R1:447-528",
                      "dims": d2_10, "two_d": True, "dtype": U8, "method": m,
                      "steps": [{"add": {"kind": "data", "w": 10, "h": 10,
                                         "data": block},
                                 "take": [[1, {"w": 5, "h": 5, "all": want}]]}]})
    # R1 test_pattern_downsampling (:626-729): 8x8 u16 gradient 100+20x+50y;
    # expectations use the test's own formulas ((v1+v2+v3+v4)/4, std::min/max)
    grad = [[100 + 20 * x + 50 * y for x in range(8)] for y in range(8)]
    exp = {MEAN: [], MIN: [], MAX: []}
    for y in range(4):
        rm, rn, rx = [], [], []
        for x in range(4):
            v = [grad[2 * y][2 * x], grad[2 * y][2 * x + 1],
                 grad[2 * y + 1][2 * x], grad[2 * y + 1][2 * x + 1]]
            rm.append(sum(v) // 4)
            rn.append(min(v))
            rx.append(max(v))
        exp[MEAN].append(rm)
        exp[MIN].append(rn)
        exp[MAX].append(rx)
    for m in (MEAN, MIN, MAX):
        cases.append({"name": f"gradient_method_{m}", "src": "R1:626-729",
                      "dims": [dim(TIME, 0, 5), dim(SPACE, 8, 4), dim(SPACE, 8, 4)],
                      "two_d": True, "dtype": U16, "method": m,
                      "steps": [{"add": {"kind": "data", "w": 8, "h": 8, "data": grad},
                                 "take": [[1, {"w": 4, "h": 4, "data": exp[m]}]]}]})
    # R1 test_3d_downsampling (:76-152): 100,200 -> 150; 100..400 -> 250 at L2
    d3 = [dim(TIME, 0, 5), dim(CHANNEL, 3, 1, 3), dim(SPACE, 20, 5),
          dim(SPACE, 20, 5), dim(SPACE, 20, 5)]
    cases.append({"name": "volume_mean_u16", "src": "R1:76-152", "dims": d3,
                  "dtype": U16, "method": MEAN,
                  "steps": [
                      {"add": const_frame(20, 20, 100), "take": [[1, None]]},
                      {"add": const_frame(20, 20, 200),
                       "take": [[1, {"w": 10, "h": 10, "all": 150}], [2, None]]},
                      {"add": const_frame(20, 20, 300), "take": [[1, None], [2, None]]},
                      {"add": const_frame(20, 20, 400),
                       "take": [[2, {"w": 5, "h": 5, "all": 250}]]}]})
    # R1 test_3d_min_max_downsampling (:530-624)
    for m, want in ((MIN, 100), (MAX, 200)):
        cases.append({"name": f"volume_pair_method_{m}", "src": "R1:552-597",
                      "dims": d3, "dtype": U16, "method": m,
                      "steps": [{"add": const_frame(20, 20, 100), "take": []},
                                {"add": const_frame(20, 20, 200),
                                 "take": [[1, {"w": 10, "h": 10, "all": want}]]}]})
    cases.append({"name": "volume_max_level2", "src": "R1:599-623", "dims": d3,
                  "dtype": U16, "method": MAX,
                  "steps": [{"add": const_frame(20, 20, v), "take": []}
                            for v in (100, 200, 300)] +
                           [{"add": const_frame(20, 20, 400),
                             "take": [[2, {"w": 5, "h": 5, "all": 400}]]}]})
    # R2 check_downsample (:88-132) x3 (:163-165): z=15, pairs on odd planes,
    # 15th plane passes through; values preserved
    dz = [dim(TIME, 0, 1), dim(SPACE, 15, 3), dim(SPACE, 48, 16), dim(SPACE, 64, 16)]
    steps = []
    for value in (63, 127, 255):
        for i in range(15):
            take = []
            if i % 2 == 1:
                take = [[1, {"w": 32, "h": 24, "all": value}]]
            if i == 14:
                take = [[1, {"w": 32, "h": 24, "all": value}]]
            steps.append({"add": const_frame(64, 48, value), "take": take})
    cases.append({"name": "odd_z_15_planes", "src": "R2:88-165", "dims": dz,
                  "dtype": U8, "method": MEAN, "steps": steps})
    # R2 test_odd_z_multi_tc_no_bleed (:19-86): t2 c2 z3, values per channel
    dn = [dim(TIME, 0, 1), dim(CHANNEL, 2, 1, 2), dim(SPACE, 3, 1),
          dim(SPACE, 8, 4), dim(SPACE, 8, 4)]
    steps = []
    for t in range(2):
        for value in (100, 200):
            for z in range(3):
                steps.append({"add": const_frame(8, 8, value), "take_any": 1})
    cases.append({"name": "odd_z_no_bleed", "src": "R2:19-86", "dims": dn,
                  "dtype": U16, "method": MEAN, "steps": steps,
                  "level1_sequence": [100, 100, 200, 200, 100, 100, 200, 200]})
    return cases


def main():
    out = {"reference": "acquire-project/acquire-zarr v0.8.1",
           "generator": "tests/golden/make_kats.py",
           "planner": planner_cases(), "stream": stream_cases()}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
