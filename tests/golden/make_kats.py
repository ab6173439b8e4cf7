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
  R4 tests/unit-tests/array-dimensions-chunk-internal-offset.cpp
  R5 tests/unit-tests/array-dimensions-tile-group-offset.cpp
  R6 tests/unit-tests/array-dimensions-chunk-lattice-index.cpp
  R7 tests/integration/stream-3d-multiscale-to-filesystem.cpp
  R8 tests/integration/stream-multiscale-trivial-3rd-dim.cpp
  R9 tests/integration/stream-2d-multiscale-to-filesystem.cpp

R4-R6 (the 203 chunk-addressing assertions) are read straight out of the
reference test files when this script runs, one fixture entry per EXPECT_EQ
line with its line number, so the fixture is a transcription, not a
computation.  R7-R9 evaluate the level expectations with the tests' own
formulas (cited per line).  The script needs /root/reference only when it is
re-run here; the tests read the committed JSON alone.

No fixture here is produced by running reference code: these are the
reference tests' own assertions, transcribed.  Fixtures made by running the
reference itself (oracle/_ref, compiled unmodified against the image's
nlohmann/json 3.1.1) are tests/golden/make_reference_vectors.py's.  The
Python package cannot be built (its pybind11 dependencies are absent).

Run: python tests/golden/make_kats.py
"""
from __future__ import annotations

import json
import os
import re

REF = "/root/reference"
DTYPE_CODES = {"uint8": 0, "uint16": 1, "uint32": 2, "uint64": 3, "int8": 4,
               "int16": 5, "int32": 6, "int64": 7, "float32": 8, "float64": 9}
DIM_TYPES = {"Space": 0, "Channel": 1, "Time": 2, "Other": 3}

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


def addressing_cases():
    """R4-R6: every EXPECT_EQ of the three ArrayDimensions addressing tests,
    with the dimensions and dtype the test builds (array.dimensions.cpp:
    232-314 is the code under test)."""
    dim_re = re.compile(r'emplace_back\(\s*"(\w+)",\s*ZarrDimensionType_(\w+),\s*(\d+),'
                        r'\s*(\d+),\s*(\d+)\)')
    dt_re = re.compile(r"ArrayDimensions dimensions\(std::move\(dims\), ZarrDataType_(\w+)\)")
    kat_re = re.compile(r"EXPECT_EQ\(int, dimensions\.(\w+)\(([\d, ]+)\), (\d+)\);")
    cases = []
    for tag, fname in (("R4", "array-dimensions-chunk-internal-offset.cpp"),
                       ("R5", "array-dimensions-tile-group-offset.cpp"),
                       ("R6", "array-dimensions-chunk-lattice-index.cpp")):
        path = os.path.join(REF, "tests", "unit-tests", fname)
        with open(path) as f:
            text = f.read()
        dims = [[DIM_TYPES[t], int(a), int(c), int(sh)]
                for _, t, a, c, sh in dim_re.findall(re.sub(r"\s+", " ", text))]
        dtype = DTYPE_CODES[dt_re.search(text).group(1)]
        asserts = []
        fn = None
        for no, line in enumerate(text.splitlines(), 1):
            m = kat_re.search(line)
            if m:
                fn = m.group(1)
                args = [int(x) for x in m.group(2).split(",")]
                asserts.append({"line": no, "args": args, "expect": int(m.group(3))})
        cases.append({"name": fname[:-4], "src": f"{tag}:{asserts[0]['line']}-"
                      f"{asserts[-1]['line']}", "function": fn, "dims": dims,
                      "dtype": dtype, "asserts": asserts})
    return cases


def integration_cases():
    """R7-R9: per-level geometry and OME scale the multiscale integration
    tests expect, evaluated with the tests' own formulas.  `frames` is the
    frame count each level receives; `scale_rule` says how the test compares
    scales (R7 compares through `EXPECT_EQ(int, ...)`, i.e. truncated)."""
    cases = []
    # R7: t10/5/2 c8/4/2 z6/2/1 (scale 1.4) y48/16/1 (0.9) x64/16/2 (0.9),
    # u16, Mean, 480 frames (:16-23, :57-125, :49-50)
    W, H, Z, C, T = 64, 48, 6, 8, 10
    cw, ch, cz, cc, ct = 16, 16, 2, 4, 5
    sw, sh, sz, sc, st = 2, 1, 1, 2, 2
    levels = []
    w, h, z, prev, acq = W, H, Z, Z, Z * C * T
    for lv in range(3):
        if lv:
            # :244-252: sizes (s+1)/2, acquired frames scaled by planes
            w, h = (w + 1) // 2, (h + 1) // 2
            prev, z = z, (z + 1) // 2
            acq = acq * z // prev
        t = -(-acq // (C * z))                                   # :254-255
        nz, ny, nx = -(-z // cz), -(-h // ch), -(-w // cw)         # :257-263
        levels.append({"sizes": [t, C, z, h, w],                    # :265-271
                       "chunks": [ct, cc, cz, ch, cw],              # chunk sizes kept
                       "shards": [st, sc, min(nz, sz), min(ny, sh), min(nx, sw)],  # :265-278
                       "scales": [1.0, 1.0, 2 ** lv * 1.4, 2 ** lv * 0.9, 2 ** lv * 0.9],
                       "frames": acq})                              # :229-233
    cases.append({"name": "stream_3d_multiscale", "src": "R7:16-23,57-125,227-278",
                  "dtype": U16, "method": MEAN, "scale_rule": "int",
                  "dims": [[TIME, T, ct, st, 1.0], [CHANNEL, C, cc, sc, 1.0],
                           [SPACE, Z, cz, sz, 1.4], [SPACE, H, ch, sh, 0.9],
                           [SPACE, W, cw, sw, 0.9]],
                  "n_levels": 3, "levels": levels})
    # R8: t5/5/1 c3/3/1 z1/1/1 (1.36) y48/16/2 (0.85) x64/16/2 (0.85), u16,
    # Mean, 15 zero frames (:16-41, :44-118); 3 datasets (:141); z scale
    # stays 1.36 (:177), y/x ~ 0.85 * (size / level size) within 0.01
    # (:182-206); level shapes are not stated by the test, only through the
    # scale relation.
    cases.append({"name": "stream_multiscale_trivial_3rd_dim",
                  "src": "R8:16-41,44-118,141,160-206", "dtype": U16, "method": MEAN,
                  "dims": [[TIME, 5, 5, 1, 1.0], [CHANNEL, 3, 3, 1, 1.0],
                           [SPACE, 1, 1, 1, 1.36], [SPACE, 48, 16, 2, 0.85],
                           [SPACE, 64, 16, 2, 0.85]],
                  "n_levels": 3, "frames_in": 15, "zero_frames": True,
                  "scale_rule": "relative_0.01",
                  "scale_relation": {"base_scale": [1.0, 1.0, 1.36, 0.85, 0.85],
                                     "fixed": [0, 1, 2], "ratio": [3, 4]}})
    # R9: t10/5/2 c8/4/2 y48/16/1 (0.9) x64/16/2 (0.9), u16, Mean, 80 frames
    # (:16-47, :50-115); per level: sizes ceil(s/2^L) (:216-221), shards
    # min(n_chunks, shard) (:223-232), scale 2^L*0.9 (:203-208)
    W, H, C, T = 64, 48, 8, 10
    levels = []
    for lv in range(3):
        w = -(-W // 2 ** lv)
        h = -(-H // 2 ** lv)
        levels.append({"sizes": [-(-80 // C), C, h, w],
                       "chunks": [5, 4, 16, 16],
                       "shards": [2, 2, min(-(-h // 16), 1), min(-(-w // 16), 2)],
                       "scales": [1.0, 1.0, 2 ** lv * 0.9, 2 ** lv * 0.9],
                       "frames": 80})
    cases.append({"name": "stream_2d_multiscale", "src": "R9:16-47,50-115,184-246",
                  "dtype": U16, "method": MEAN, "scale_rule": "exact",
                  "dims": [[TIME, T, 5, 2, 1.0], [CHANNEL, C, 4, 2, 1.0],
                           [SPACE, H, 16, 1, 0.9], [SPACE, W, 16, 2, 0.9]],
                  "n_levels": 3, "levels": levels})
    return cases


def main():
    out = {"reference": "acquire-project/acquire-zarr v0.8.1",
           "generator": "tests/golden/make_kats.py",
           "planner": planner_cases(), "stream": stream_cases(),
           "addressing": addressing_cases(), "integration": integration_cases()}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
