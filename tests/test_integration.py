"""CPU: the acquire-zarr drop-in (integration/) against the reference's own
tree — VERDICT r1 items 1 and 7.

In a scratch copy of /root/reference (never written to), integration/apply.sh
applies acquire-zarr-hip.patch and installs cmake/hip.cmake plus the two new
src/streaming sources.  Then:

* the patched downsampler.cpp, the adapter downsampler.hip.cpp and the
  sources they need are compiled with -DAQZ_DOWNSAMPLER_HIP against the
  reference's headers and linked against libaqz_downsampler.so, every aqz_
  symbol resolving there and nothing else unresolved but three helpers of
  zarr.common.cpp (which needs blosc/zstd headers): the zarr::Downsampler
  contract (downsampler.hh:11-64) is met by the C ABI;
* the patched multiscale.array.cpp (overlap + tiled takes) and array.tiled.cpp
  are compiled (syntax/semantic check; their link needs the whole library);
* the default CPU build of the patched downsampler.cpp still compiles;
* cmake/hip.cmake configures a toy target for AQZ_DOWNSAMPLER=hip/cpu and
  rejects anything else.

* the patched array.cpp (its three tiled-frame hooks) compiles in both modes;
* the tiled chunk writer (array.tiled.cpp) RUNS on the reference's own
  ArrayDimensions and Chunk (array.dimensions.cpp, chunk.cpp, zarr.common.cpp,
  compiled from /root/reference): chunk bytes, has_data and the bytes written
  per frame must equal what write_frame_to_chunks_ (array.cpp:507-622) leaves
  — the oracle's tiling placed by the oracle's KAT-pinned addressing — on
  ragged frames, several layers and N-D chunk lattices.

nlohmann/json is the image's genuine 3.1.1 (/opt/conda/include/json.hpp,
reached as <nlohmann/json.hpp> through a symlink); blosc.h and zstd.h are the
image's own (/opt/conda/include).  google/crc32c is not in this image:
tests/integration/crc32c/crc32c.h declares its one entry point so the patched
array.cpp can be syntax-checked, and nothing built with it is linked or run.
The adapter itself is linked here and EXECUTED on the GPU by
tests/test_gpu_adapter.py (tests/integration/build_adapter_harness.sh).
Skipped when /root/reference is absent (the GPU box)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
STUB = os.path.join(ROOT, "tests", "integration")
LIB_DIR = os.path.join(ROOT, "acquire-zarr_amd")
CONDA_INC = "/opt/conda/include"   # blosc.h, zstd.h (part of the image)
CONDA_LIB = "/opt/conda/lib"
JSON_HPP = "/opt/conda/include/json.hpp"  # nlohmann/json 3.1.1, part of the image

pytestmark = pytest.mark.skipif(
    not os.path.exists(os.path.join(REF, "src", "streaming", "downsampler.hh")),
    reason="reference tree absent (integration check runs in the build container)")


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    t = tmp_path_factory.mktemp("acquire-zarr")
    inc = t / "_json_inc" / "nlohmann"
    inc.mkdir(parents=True)
    os.symlink(JSON_HPP, inc / "json.hpp")
    for d in ("include", "cmake", os.path.join("src", "streaming"), os.path.join("src", "logger")):
        shutil.copytree(os.path.join(REF, d), t / d)
    shutil.copy(os.path.join(REF, "CMakeLists.txt"), t / "CMakeLists.txt")
    r = subprocess.run([os.path.join(ROOT, "integration", "apply.sh"), str(t)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert not list(t.rglob("*.rej")), "patch hunks rejected"
    return t


def gxx(tree, args, defines=("AQZ_DOWNSAMPLER_HIP",)):
    cmd = ["g++", "-std=c++20", "-fPIC", "-Wall", "-Wno-unknown-pragmas",
           "-Wno-sign-compare", "-Wno-unused-variable"]
    cmd += [f"-D{d}" for d in defines]
    cmd += ["-I", str(tree / "_json_inc"), "-I", STUB, "-I", os.path.join(ROOT, "include"),
            "-I", str(tree / "include"), "-I", str(tree / "src" / "streaming"),
            "-I", str(tree / "src" / "logger"), "-idirafter", CONDA_INC] + list(args)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, " ".join(cmd) + "\n" + r.stderr[-4000:]
    return r


def test_patch_applies_and_keeps_reference_bodies_out(tree):
    s = (tree / "src" / "streaming" / "downsampler.cpp").read_text()
    # the CPU per-frame path is compiled out in the HIP build, the planner and
    # metadata stay (they are the reference's own code)
    assert s.count("#ifndef AQZ_DOWNSAMPLER_HIP") == 2
    assert "make_writer_configurations_" in s and "get_metadata" in s
    a = (tree / "src" / "streaming" / "array.cpp").read_text()
    assert "return write_tiles_to_chunks_(frame);" in a
    assert "tiled_ ? bytes_of_frame(*config_->dimensions, config_->dtype)" in a
    # the Ok/PartialWrite result compares with the payload, not the tiled
    # buffer's size (which includes the zero overhang)
    assert "return bytes_written == nbytes_data ? WriteResult::Ok" in a
    top = (tree / "CMakeLists.txt").read_text()
    assert "include(cmake/hip.cmake)" in top
    streaming = (tree / "src" / "streaming" / "CMakeLists.txt").read_text()
    i, j = (streaming.index("target_enable_simd(${tgt})"),
            streaming.index("target_enable_hip_downsampler(${tgt})"))
    assert i < j
    # the committed adapter sources carry no reference function bodies
    for f in ("downsampler.hip.cpp", "array.tiled.cpp"):
        src = open(os.path.join(ROOT, "integration", "src", "streaming", f)).read()
        for ref_only in ("scale_image", "average_two_frames", "write_frame_to_chunks_(std",
                         "downscale_local_mean", "partial_scaled_frames_"):
            assert ref_only not in src, (f, ref_only)


def test_adapter_links_against_the_c_abi(tree, tmp_path):
    lib = os.path.join(LIB_DIR, "libaqz_downsampler.so")
    assert os.path.exists(lib), "build the library first (__graft_entry__.build())"
    srcs = [tree / "src" / "streaming" / "downsampler.cpp",
            tree / "src" / "streaming" / "downsampler.hip.cpp",
            tree / "src" / "streaming" / "array.dimensions.cpp",
            tree / "src" / "streaming" / "zarr.common.cpp",
            tree / "src" / "logger" / "logger.cpp"]
    objs = []
    for s in srcs:
        o = tmp_path / (s.stem + ".o")
        gxx(tree, ["-O1", "-c", str(s), "-o", str(o)])
        objs.append(str(o))
    # Every symbol the adapter needs resolves in libaqz_downsampler.so, the
    # reference's own objects, the image's c-blosc / zstd or the C/C++ runtime.
    libs = tmp_path / "lib"
    libs.mkdir()
    for name in ("libblosc.so.1", "liblz4.so.1", "libz.so.1", "libzstd.so.1"):
        shutil.copy(os.path.join(CONDA_LIB, name), libs / name)
    os.symlink("libblosc.so.1", libs / "libblosc.so")
    os.symlink("libzstd.so.1", libs / "libzstd.so")
    so = tmp_path / "libzarr_downsampler_hip.so"
    gxx(tree, ["-shared", "-o", str(so)] + objs +
        ["-L", LIB_DIR, "-laqz_downsampler", f"-Wl,-rpath,{LIB_DIR}",
         "-L", str(libs), "-lblosc", "-lzstd", f"-Wl,-rpath,{libs}",
         "-Wl,-rpath,/opt/rocm/lib", "-lpthread"])
    undef = subprocess.run(["nm", "-DC", "--undefined-only", str(so)],
                           capture_output=True, text=True, check=True).stdout.splitlines()
    exported = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True,
                              text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in exported.splitlines() if ln.strip()}
    unresolved = set()
    for ln in undef:
        name = ln.split(None, 1)[1].strip()
        if ln.split()[0] == "w" or "@" in name:  # weak, or versioned libc/libstdc++
            continue
        if name.startswith("aqz_"):
            assert name in exported, f"{name} not exported by libaqz_downsampler.so"
            continue
        if name.startswith(("blosc_", "ZSTD_")):
            continue
        unresolved.add(name)
    assert not unresolved, unresolved
    nm = "\n".join(undef)
    for sym in ("aqz_ds_create", "aqz_ds_add_frame", "aqz_ds_add_frame_async_take",
                "aqz_ds_wait", "aqz_ds_take_frame", "aqz_ds_take_frame_tiled",
                "aqz_ds_set_level_tiling", "aqz_ds_destroy"):
        assert sym in nm, sym
    defined = subprocess.run(["nm", "-DC", "--defined-only", str(so)],
                             capture_output=True, text=True, check=True).stdout
    for m in ("zarr::Downsampler::Downsampler(", "zarr::Downsampler::~Downsampler()",
              "zarr::Downsampler::add_frame(", "zarr::Downsampler::take_frame(",
              "zarr::Downsampler::add_frame_async(", "zarr::Downsampler::take_frame_tiled(",
              "zarr::Downsampler::get_metadata",
              "zarr::Downsampler::writer_configurations() const"):
        assert m in defined, m


def test_callers_compile(tree):
    # MultiscaleArray::write_frame reordered (add_frame_async before level 0's
    # chunking, tiled takes for levels >= 1) and Array's tiled write
    for f in ("multiscale.array.cpp", "array.tiled.cpp"):
        gxx(tree, ["-fopenmp", "-fsyntax-only", str(tree / "src" / "streaming" / f)])


def test_cpu_build_unchanged(tree):
    # AQZ_DOWNSAMPLER=cpu: the patched files compile to the reference's code
    for f in ("downsampler.cpp", "multiscale.array.cpp", "array.cpp"):
        gxx(tree, ["-fopenmp", "-fsyntax-only", str(tree / "src" / "streaming" / f)],
            defines=())


def test_patched_array_cpp_compiles(tree):
    # the three hooks (payload size, Ok/PartialWrite, tiled dispatch) in the
    # HIP build of the reference's own array.cpp
    gxx(tree, ["-fopenmp", "-fsyntax-only", str(tree / "src" / "streaming" / "array.cpp")])


@pytest.fixture(scope="module")
def harness(tree, tmp_path_factory):
    """tests/integration/tiled_writer_harness.cpp linked with the reference's
    array.dimensions.cpp, chunk.cpp, zarr.common.cpp and logger.cpp and the
    drop-in's array.tiled.cpp (placement only)."""
    out = tmp_path_factory.mktemp("harness")
    # libblosc's RPATH is $ORIGIN: a private copy with its codecs keeps
    # /opt/conda/lib (and its older libstdc++) off the harness's search path
    libs = out / "lib"
    libs.mkdir()
    for name in ("libblosc.so.1", "liblz4.so.1", "libz.so.1", "libzstd.so.1"):
        shutil.copy(os.path.join(CONDA_LIB, name), libs / name)
    os.symlink("libblosc.so.1", libs / "libblosc.so")
    os.symlink("libzstd.so.1", libs / "libzstd.so")
    srcs = [tree / "src" / "streaming" / "array.dimensions.cpp",
            tree / "src" / "streaming" / "chunk.cpp",
            tree / "src" / "streaming" / "zarr.common.cpp",
            tree / "src" / "logger" / "logger.cpp",
            tree / "src" / "streaming" / "array.tiled.cpp",
            os.path.join(STUB, "tiled_writer_harness.cpp")]
    exe = out / "tiled_writer_harness"
    gxx(tree, ["-O1", "-fopenmp", "-DAQZ_TILED_STANDALONE", "-o", str(exe)] +
        [str(x) for x in srcs] + ["-L", str(libs), "-lblosc", "-lzstd", f"-Wl,-rpath,{libs}",
                                  "-lpthread"], defines=())
    return exe


SPACE, CHANNEL, TIME = 0, 1, 2


def _run_harness(exe, tmp_path, oracle, dims, dtype, n_frames, seed):
    import numpy as np
    np_dt = np.dtype(dtype)
    bpp = np_dt.itemsize
    H, W = dims[-2][1], dims[-1][1]
    tr, tc = dims[-2][2], dims[-1][2]
    rng = np.random.default_rng(seed)
    frames = rng.integers(1, 200, (n_frames, H, W)).astype(dtype)
    frames[1::3, :tr, :] = 0            # whole zero tile rows in some frames
    if n_frames > 4:
        frames[4] = 0                   # and one all-zero frame
    tiles = [oracle.tile_frame(f, tr, tc)[0] for f in frames]
    blob = b"".join(t.tobytes() for t in tiles)
    (tmp_path / "tiles.bin").write_bytes(blob)
    spec = f"{len(dims)} {bpp} {oracle.dtype_code(dtype)} {n_frames}\n" + \
        "".join(f"{t} {a} {c} {s}\n" for t, a, c, s in dims)
    r = subprocess.run([str(exe), str(tmp_path / "tiles.bin"), str(tmp_path / "chunks.bin")],
                       input=spec, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    written = [int(ln.split()[2]) for ln in r.stdout.splitlines() if ln.startswith("frame ")]
    # what the patched write_frame compares with: one frame's payload, so a
    # ragged level returns WriteResult::Ok, never PartialWrite
    assert written == [H * W * bpp] * n_frames
    # expected chunk layers: the oracle's tiles at the oracle's offsets
    # (array.dimensions.cpp:232-314, pinned to the reference's KATs)
    offs, cb, lb = oracle.chunk_frame_offsets(dims, bpp, 0, n_frames)
    n_layers = max(offs) // lb + 1
    want = np.zeros(n_layers * lb, np.uint8)
    touched = np.zeros(n_layers * (lb // cb), bool)
    tb = tr * tc * bpp
    for k in range(n_frames):
        for t in range(tiles[k].shape[0]):
            at = offs[k] + t * cb
            want[at:at + tb] = tiles[k][t].view(np.uint8).reshape(-1)
            touched[at // cb] = True
    got = np.frombuffer((tmp_path / "chunks.bin").read_bytes(), np.uint8)
    assert got.size == n_layers * (lb // cb) * (cb + 1)
    got = got.reshape(-1, cb + 1)
    state, data = got[:, 0], got[:, 1:].reshape(-1)
    np.testing.assert_array_equal(data, want)
    want_state = np.where(~touched, 0,
                          np.where(want.reshape(-1, cb).any(axis=1), 2, 1))
    np.testing.assert_array_equal(state, want_state)
    return written


@pytest.mark.parametrize("dims,dtype,n", [
    # T/Y/X, ragged level (the 3000x3000 shape class: not a multiple of the
    # chunk), 3 frames per chunk, 3 layers with a partial last one
    ([(TIME, 0, 3, 1), (SPACE, 75, 32, 1), (SPACE, 93, 32, 1)], "uint16", 8),
    # the reference's addressing-test dims (t 0/5, c 3/2, z 5/2, y 48/16,
    # x 64/16): all 76 frames its KATs name, the 76th opens layer 2
    ([(TIME, 0, 5, 1), (CHANNEL, 3, 2, 1), (CHANNEL, 5, 2, 1), (SPACE, 48, 16, 1),
      (SPACE, 64, 16, 1)], "uint16", 76),
    # T/C/Y/X with ragged XY and channels chunked 2 of 3, f32
    ([(TIME, 0, 2, 1), (CHANNEL, 3, 2, 1), (SPACE, 40, 16, 1), (SPACE, 37, 16, 1)],
     "float32", 9),
    # single-tile frames narrower than a chunk, u8
    ([(TIME, 0, 4, 1), (SPACE, 7, 8, 1), (SPACE, 5, 8, 1)], "uint8", 6),
])
def test_tiled_writer_runs_on_reference_chunks(harness, tmp_path, oracle, dims, dtype, n):
    import numpy as np
    _run_harness(harness, tmp_path, oracle, dims, np.dtype(dtype), n, seed=len(dims) + n)


def _configure(tree, tmp_path, value):
    proj = tmp_path / f"toy_{value}"
    proj.mkdir()
    for f in ("downsampler.hip.cpp", "array.tiled.cpp"):
        shutil.copy(tree / "src" / "streaming" / f, proj / f)
    (proj / "stub.cpp").write_text("int aqz_toy() { return 0; }\n")
    (proj / "CMakeLists.txt").write_text(
        "cmake_minimum_required(VERSION 3.20)\n"
        "project(aqz_hip_cmake_check CXX)\n"
        f"include({tree}/cmake/hip.cmake)\n"
        "add_library(toy OBJECT stub.cpp)\n"
        "target_enable_hip_downsampler(toy)\n"
        "get_target_property(srcs toy SOURCES)\n"
        "get_target_property(defs toy COMPILE_DEFINITIONS)\n"
        "message(STATUS \"toy sources: ${srcs}; defs: ${defs}\")\n")
    return subprocess.run(["cmake", "-S", str(proj), "-B", str(proj / "build"),
                           f"-DAQZ_DOWNSAMPLER={value}", f"-DAQZ_DS_ROOT={ROOT}"],
                          capture_output=True, text=True, timeout=300)


def test_hip_cmake_configures(tree, tmp_path):
    r = _configure(tree, tmp_path, "hip")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "multiscale downsampler on MI355X" in r.stdout
    assert "downsampler.hip.cpp" in r.stdout and "array.tiled.cpp" in r.stdout
    assert "AQZ_DOWNSAMPLER_HIP" in r.stdout
    r = _configure(tree, tmp_path, "cpu")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "downsampler.hip.cpp" not in r.stdout
    r = _configure(tree, tmp_path, "cuda")
    assert r.returncode != 0 and "must be 'cpu' or 'hip'" in (r.stdout + r.stderr)
