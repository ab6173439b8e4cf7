"""Regenerate the fixtures made by the REFERENCE ITSELF (tests/refvec.py):

    make -C oracle ref                                   # builds oracle/_ref
    python tests/golden/make_reference_vectors.py        # vectors + manifest
    python tests/golden/make_reference_vectors.py --digests   # + BASELINE digests
    python tests/golden/make_reference_vectors.py --nan-only  # NaN-payload set only

Every output byte here comes from acquire-zarr v0.8.1's own
zarr::Downsampler / ArrayDimensions (src/streaming/downsampler.cpp,
array.dimensions.cpp), compiled unmodified from /root/reference by
oracle/Makefile and called through oracle/ref_shim.cpp.  Nothing is computed
by the oracle or the product.  Needs the reference tree (this container);
the committed fixtures travel, the reference does not.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import digest_util as du  # noqa: E402
import ref  # noqa: E402  (oracle/ref.py: the reference's own code)
import refvec as rv  # noqa: E402

SEED = 0x5EF0C0DE


def vectors():
    man = {"made_by": "acquire-zarr v0.8.1 src/streaming/downsampler.cpp (unmodified, "
                      "oracle/_ref via oracle/ref_shim.cpp) — tests/golden/"
                      "make_reference_vectors.py",
           "nlohmann_json": "3.1.1 (/opt/conda/include/json.hpp, the image's)",
           "dtypes": [np.dtype(t).name for t in rv.NP_DTYPES],
           "geometries": {}, "methods": {}, "errors": {}}
    arrays = {}
    for gi, (geom, (dims, n_frames, take)) in enumerate(rv.GEOMETRIES.items()):
        entry = {"dims": dims, "frames": n_frames, "take": take}
        for di, dt in enumerate(rv.NP_DTYPES):
            dname = np.dtype(dt).name
            x = rv.make_inputs(geom, dt, SEED + 100 * gi + di)
            arrays[f"in/{geom}/{dname}"] = x
            for m in range(4):
                ds = ref.RefDownsampler(dims, dt, m)
                if "levels" not in entry:
                    entry["levels"] = ds.levels
                    entry["geometry"] = ds.geometry
                assert ds.levels == entry["levels"]
                ev, out = [], []
                for k in range(n_frames):
                    ds.add_frame(x[k])
                    if not rv.take_now(take, k):
                        continue
                    for L in range(1, ds.n_levels):
                        b = ds.take_bytes(L)
                        ev.append((k, L, b is not None, 0 if b is None else b.size))
                        if b is not None:
                            out.append(b)
                name = rv.case_name(geom, dt, m)
                arrays[f"ev/{name}"] = np.array(ev, dtype=np.int64).reshape(-1, 4)
                arrays[f"out/{name}"] = (np.concatenate(out) if out
                                         else np.zeros(0, np.uint8))
        man["geometries"][geom] = entry
        print(geom, entry["geometry"], flush=True)
    dims = rv.GEOMETRIES["xy_odd_37x29"][0]
    for m in range(4):
        ds = ref.RefDownsampler(dims, np.uint16, m)
        man["methods"][rv.METHOD_NAMES[m]] = {"downsampling_method": ds.downsampling_method(),
                                              "get_metadata": ds.metadata_json()}
    # the reference's own messages for an invalid dtype (Downsampler ctor,
    # downsampler.cpp:293-295) and method (ArrayConfig ctor, array.base.hh:36-41)
    for what, dt_code, m in (("dtype", 10, 1), ("method", 0, 4)):
        err = ctypes.create_string_buffer(512)
        h = ref.lib().ref_ds_create(ref._dims(dims), len(dims), dt_code, m, 0, err, len(err))
        assert not h, what
        man["errors"][what] = {"dtype": dt_code, "method": m, "message": err.value.decode()}
    np.savez_compressed(rv.NPZ, **arrays)
    with open(rv.MANIFEST, "w") as f:
        json.dump(man, f, indent=1)
        f.write("\n")
    print("wrote", rv.NPZ, os.path.getsize(rv.NPZ), "bytes")


def nan_vectors():
    """The NaN-payload cases (refvec.NAN_GEOMETRIES x float dtypes x methods),
    same layout as the main vectors; geometries come from the main manifest."""
    arrays = {}
    for gi, geom in enumerate(rv.NAN_GEOMETRIES):
        dims, n_frames, take = rv.GEOMETRIES[geom]
        for di, dt in enumerate(rv.NAN_DTYPES):
            dname = np.dtype(dt).name
            x = rv.make_nan_inputs(geom, dt, SEED + 7000 + 100 * gi + di)
            arrays[f"in/{geom}/{dname}"] = x
            for m in range(4):
                ds = ref.RefDownsampler(dims, dt, m)
                ev, out = [], []
                for k in range(n_frames):
                    ds.add_frame(x[k])
                    if not rv.take_now(take, k):
                        continue
                    for L in range(1, ds.n_levels):
                        b = ds.take_bytes(L)
                        ev.append((k, L, b is not None, 0 if b is None else b.size))
                        if b is not None:
                            out.append(b)
                name = rv.case_name(geom, dt, m)
                arrays[f"ev/{name}"] = np.array(ev, dtype=np.int64).reshape(-1, 4)
                arrays[f"out/{name}"] = (np.concatenate(out) if out
                                         else np.zeros(0, np.uint8))
    np.savez_compressed(rv.NAN_NPZ, **arrays)
    print("wrote", rv.NAN_NPZ, os.path.getsize(rv.NAN_NPZ), "bytes")


def digests():
    out = {"generator": "tests/digest_util.py (splitmix64, seed 0xA0C2A11 + sorted config index)",
           "digest": "sha256 of each level's taken frames, concatenated in order",
           "made_by": "acquire-zarr v0.8.1 zarr::Downsampler (oracle/_ref, unmodified "
                      "reference sources) via tests/golden/make_reference_vectors.py --digests",
           "configs": {}}

    def make_ref(dims, dtype, method):
        ds = ref.RefDownsampler(dims, dtype, method)
        return ds, ds.geometry

    for name in du.CONFIGS:
        dims, dtype, frames = du.CONFIGS[name]
        entry = {"dims": dims, "dtype": np.dtype(dtype).name, "frames": frames, "methods": {}}
        for m, mname in enumerate(du.METHOD_NAMES):
            t = time.time()
            entry["methods"][mname] = du.run_stream(make_ref, name, m)
            print(name, mname, f"{time.time() - t:.1f}s", flush=True)
        out["configs"][name] = entry
    with open(rv.DIGESTS, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--digests", action="store_true", help="also the BASELINE-config digests")
    ap.add_argument("--nan-only", action="store_true",
                    help="only the NaN-payload vectors (reference_nan_vectors.npz)")
    a = ap.parse_args()
    if not ref.build():
        sys.exit("oracle/_ref is not built and /root/reference is absent")
    nan_vectors()
    if a.nan_only:
        return
    vectors()
    if a.digests:
        digests()


if __name__ == "__main__":
    main()
