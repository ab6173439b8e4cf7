"""ctypes front-end of the CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker.  The product path
(acquire-zarr_amd/) never imports it.

The C restatement lives in ds_oracle.c (acquire-zarr v0.8.1
src/streaming/downsampler.cpp, cited per function there).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_ds.so")

# numpy dtypes indexed by ZarrDataType value (zarr.types.h:55-68)
NP_DTYPES = [np.uint8, np.uint16, np.uint32, np.uint64, np.int8, np.int16,
             np.int32, np.int64, np.float32, np.float64]
DTYPE_BY_NAME = {np.dtype(t).name: i for i, t in enumerate(NP_DTYPES)}

DECIMATE, MEAN, MIN, MAX = 0, 1, 2, 3
SPACE, CHANNEL, TIME, OTHER = 0, 1, 2, 3


class Dim(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32),
                ("array_size_px", ctypes.c_uint32),
                ("chunk_size_px", ctypes.c_uint32),
                ("shard_size_chunks", ctypes.c_uint32),
                ("scale", ctypes.c_double)]


def build() -> str:
    """Compile the oracle with its Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32
        L.oracle_scale_image.argtypes = [ctypes.c_int, ctypes.c_int, vp, sz, sz, vp]
        L.oracle_average_two_frames.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, sz]
        L.oracle_reduce4.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp]
        L.oracle_reduce2.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp]
        L.oracle_plan_levels.argtypes = [ctypes.POINTER(Dim), u32, u32,
                                         ctypes.POINTER(Dim), u32,
                                         ctypes.POINTER(u32)]
        L.oracle_ds_create.restype = vp
        L.oracle_ds_create.argtypes = [ctypes.POINTER(u32)] * 3 + [u32, ctypes.c_int, ctypes.c_int]
        L.oracle_ds_destroy.argtypes = [vp]
        L.oracle_ds_add_frame.argtypes = [vp, vp, sz]
        L.oracle_ds_take_frame.argtypes = [vp, u32, vp, sz, ctypes.POINTER(sz)]
        L.oracle_tile_frame.argtypes = [ctypes.c_int, vp, u32, u32, u32, u32, vp, vp]
        L.oracle_transpose_frame.argtypes = [ctypes.c_int, vp, u32, u32, vp]
        L.oracle_blosc_filter.argtypes = [ctypes.c_int, u32, u32, vp, sz, vp, vp]
        L.oracle_blosc_unfilter.argtypes = [ctypes.c_int, u32, u32, vp, sz, vp]
        L.oracle_crc32c.argtypes = [vp, sz]
        L.oracle_crc32c.restype = u32
        L.oracle_shard_index_table.argtypes = [vp, vp, sz, vp]
        L.oracle_ds_level_count.argtypes = [vp, u32]
        L.oracle_ds_level_count.restype = u32
        u64 = ctypes.c_uint64
        L.oracle_chunk_lattice_index.argtypes = [ctypes.POINTER(Dim), u32, u64, u32]
        L.oracle_chunk_lattice_index.restype = u32
        L.oracle_tile_group_offset.argtypes = [ctypes.POINTER(Dim), u32, u64]
        L.oracle_tile_group_offset.restype = u64
        L.oracle_chunk_internal_offset.argtypes = [ctypes.POINTER(Dim), u32, u32, u64]
        L.oracle_chunk_internal_offset.restype = u64
        _lib = L
    return _lib


def dtype_code(dt) -> int:
    return DTYPE_BY_NAME[np.dtype(dt).name]


def scale_image(img: np.ndarray, method: int) -> np.ndarray:
    """One 2x2 level (scale_image<T>, downsampler.cpp:139-206)."""
    img = np.ascontiguousarray(img)
    h, w = img.shape
    out = np.zeros(((h + h % 2) // 2, (w + w % 2) // 2), dtype=img.dtype)
    rc = lib().oracle_scale_image(dtype_code(img.dtype), method,
                                  img.ctypes.data, w, h, out.ctypes.data)
    if rc:
        raise ValueError("oracle_scale_image failed")
    return out


def average_two_frames(earlier: np.ndarray, current: np.ndarray, method: int) -> np.ndarray:
    """average_two_frames<T> (downsampler.cpp:208-246): f(earlier, current)."""
    dst = np.ascontiguousarray(earlier).copy()
    src = np.ascontiguousarray(current)
    assert dst.shape == src.shape and dst.dtype == src.dtype
    rc = lib().oracle_average_two_frames(dtype_code(dst.dtype), method,
                                         dst.ctypes.data, src.ctypes.data, dst.size)
    if rc:
        raise ValueError("oracle_average_two_frames failed")
    return dst


def reduce4(dt, method, a, b, c, d):
    v = np.array([a, b, c, d], dtype=dt)
    out = np.zeros(1, dtype=dt)
    p = v.ctypes.data
    isz = v.itemsize
    lib().oracle_reduce4(dtype_code(dt), method, p, p + isz, p + 2 * isz, p + 3 * isz,
                         out.ctypes.data)
    return out[0]


def reduce2(dt, method, a, b):
    v = np.array([a, b], dtype=dt)
    out = np.zeros(1, dtype=dt)
    lib().oracle_reduce2(dtype_code(dt), method, v.ctypes.data,
                         v.ctypes.data + v.itemsize, out.ctypes.data)
    return out[0]


def plan_levels(dims, max_levels: int = 0):
    """make_writer_configurations_ (downsampler.cpp:493-597).

    `dims` is a list of (type, array_size, chunk_size, shard_size[, scale])
    tuples in storage order with ndims >= 3 (2-D arrays get the phantom
    singleton dim first, array.dimensions.cpp:149-152).  Returns a list of
    levels, each a list of (type, size, chunk, shard, scale) tuples.
    """
    nd = len(dims)
    arr = (Dim * nd)(*[Dim(d[0], d[1], d[2], d[3], d[4] if len(d) > 4 else 1.0) for d in dims])
    n = ctypes.c_uint32(0)
    rc = lib().oracle_plan_levels(arr, nd, max_levels, None, 0, ctypes.byref(n))
    if rc:
        raise ValueError("oracle_plan_levels failed")
    out = (Dim * (nd * n.value))()
    rc = lib().oracle_plan_levels(arr, nd, max_levels, out, n.value, ctypes.byref(n))
    if rc:
        raise ValueError("oracle_plan_levels failed")
    return [[(o.type, o.array_size_px, o.chunk_size_px, o.shard_size_chunks, o.scale)
             for o in out[l * nd:(l + 1) * nd]] for l in range(n.value)]


def level_geometry(levels):
    """(width, height, planes) per level, as Downsampler::add_frame reads them."""
    return [(lv[-1][1], lv[-2][1], lv[-3][1]) for lv in levels]


class OracleDownsampler:
    """Downsampler::add_frame / take_frame (downsampler.cpp:306-414)."""

    def __init__(self, geometry, dtype, method):
        self.dtype = np.dtype(dtype)
        self.geometry = list(geometry)
        n = len(self.geometry)
        W = (ctypes.c_uint32 * n)(*[g[0] for g in self.geometry])
        H = (ctypes.c_uint32 * n)(*[g[1] for g in self.geometry])
        P = (ctypes.c_uint32 * n)(*[g[2] for g in self.geometry])
        self._h = lib().oracle_ds_create(W, H, P, n, dtype_code(self.dtype), method)
        if not self._h:
            raise ValueError("invalid oracle downsampler arguments")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().oracle_ds_destroy(h)
            self._h = None

    def add_frame(self, frame: np.ndarray):
        frame = np.ascontiguousarray(frame, dtype=self.dtype)
        rc = lib().oracle_ds_add_frame(self._h, frame.ctypes.data, frame.nbytes)
        if rc:
            raise RuntimeError("oracle add_frame: frame size mismatch")

    def take_frame(self, level: int):
        w, h, _ = self.geometry[level]
        out = np.empty((h, w), dtype=self.dtype)
        nb = ctypes.c_size_t(0)
        rc = lib().oracle_ds_take_frame(self._h, level, out.ctypes.data, out.nbytes,
                                        ctypes.byref(nb))
        if rc < 0:
            raise RuntimeError("oracle take_frame failed")
        return out if rc == 1 else None

    def level_count(self, level: int) -> int:
        return lib().oracle_ds_level_count(self._h, level)


def tile_frame(img: np.ndarray, tile_rows: int, tile_cols: int):
    """Chunk tiling of one frame (array.cpp:507-622, chunk.cpp:17-58):
    returns (tiles[n_tiles, tile_rows, tile_cols], nonzero[n_tiles])."""
    img = np.ascontiguousarray(img)
    h, w = img.shape
    nty, ntx = -(-h // tile_rows), -(-w // tile_cols)
    out = np.empty((nty * ntx, tile_rows, tile_cols), dtype=img.dtype)
    nz = np.empty(nty * ntx, dtype=np.uint8)
    rc = lib().oracle_tile_frame(dtype_code(img.dtype), img.ctypes.data, w, h,
                                 tile_rows, tile_cols, out.ctypes.data, nz.ctypes.data)
    if rc:
        raise ValueError("oracle_tile_frame failed")
    return out, nz.astype(bool)


def transpose_frame(img: np.ndarray):
    """transpose_frame (array.cpp:488-504) of a rows x cols frame."""
    img = np.ascontiguousarray(img)
    rows, cols = img.shape
    out = np.empty((cols, rows), dtype=img.dtype)
    if lib().oracle_transpose_frame(dtype_code(img.dtype), img.ctypes.data, rows, cols,
                                    out.ctypes.data):
        raise ValueError("oracle_transpose_frame failed")
    return out


def blosc_filter(buf, shuffle: int, typesize: int, blocksize: int) -> np.ndarray:
    """Bytes c-blosc feeds its codec, block by block (codec_oracle.c)."""
    src = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    out = np.empty_like(src)
    tmp = np.empty(max(blocksize, 1), np.uint8)
    if lib().oracle_blosc_filter(shuffle, typesize, blocksize, src.ctypes.data, src.size,
                                 out.ctypes.data, tmp.ctypes.data):
        raise ValueError("oracle_blosc_filter: bad arguments")
    return out


def blosc_unfilter(buf, shuffle: int, typesize: int, blocksize: int) -> np.ndarray:
    src = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    out = np.empty_like(src)
    if lib().oracle_blosc_unfilter(shuffle, typesize, blocksize, src.ctypes.data, src.size,
                                   out.ctypes.data):
        raise ValueError("oracle_blosc_unfilter: bad arguments")
    return out


def crc32c(buf) -> int:
    b = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    return int(lib().oracle_crc32c(b.ctypes.data, b.size))


def shard_index_table(offsets, extents) -> np.ndarray:
    """Shard::write_table_ (shard.cpp:145-166) bytes: pairs then crc32c."""
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ext = np.ascontiguousarray(extents, dtype=np.uint64)
    out = np.empty(16 * off.size + 4, np.uint8)
    lib().oracle_shard_index_table(off.ctypes.data, ext.ctypes.data, off.size,
                                   out.ctypes.data)
    return out


def cascade_2d(frame: np.ndarray, n_levels: int, method: int):
    """Pure XY pyramid of `n_levels` total levels (levels 1..n-1 returned)."""
    out = []
    cur = frame
    for _ in range(1, n_levels):
        cur = scale_image(cur, method)
        out.append(cur)
    return out


def _dim_array(dims):
    return (Dim * len(dims))(*[Dim(d[0], d[1], d[2], d[3], d[4] if len(d) > 4 else 1.0)
                               for d in dims])


def chunk_lattice_index(dims, frame_id: int, dim_index: int) -> int:
    """ArrayDimensions::chunk_lattice_index (array.dimensions.cpp:232-262)."""
    r = lib().oracle_chunk_lattice_index(_dim_array(dims), len(dims), frame_id, dim_index)
    if r == 0xFFFFFFFF:
        raise ValueError("invalid dimension index")
    return int(r)


def tile_group_offset(dims, frame_id: int) -> int:
    """ArrayDimensions::tile_group_offset (array.dimensions.cpp:264-282), in chunks."""
    return int(lib().oracle_tile_group_offset(_dim_array(dims), len(dims), frame_id))


def chunk_internal_offset(dims, bytes_per_px: int, frame_id: int) -> int:
    """ArrayDimensions::chunk_internal_offset (array.dimensions.cpp:284-314), in bytes."""
    return int(lib().oracle_chunk_internal_offset(_dim_array(dims), len(dims), bytes_per_px,
                                                  frame_id))


def chunk_frame_offsets(dims, bytes_per_px: int, first_frame: int, n_frames: int):
    """Where each frame's tile 0 lands in a buffer of whole chunk layers,
    relative to first_frame's layer: (offsets, chunk_bytes, layer_bytes).

    Array::write_frame_to_chunks_ (array.cpp:563-617) writes tile t of frame
    k into chunks_[t + tile_group_offset(k)] at chunk_internal_offset(k); one
    layer holds number_of_chunks_in_memory_ chunks of bytes_per_chunk_
    (array.dimensions.cpp:168-178); chunk_lattice_index(k, 0) is the layer.
    """
    chunk_bytes = bytes_per_px
    for d in dims:
        chunk_bytes *= d[2]
    layer_chunks = 1
    for d in dims[1:]:
        layer_chunks *= -(-d[1] // d[2])
    layer_bytes = layer_chunks * chunk_bytes
    base = chunk_lattice_index(dims, first_frame, 0)
    offs = []
    for k in range(first_frame, first_frame + n_frames):
        layer = chunk_lattice_index(dims, k, 0) - base
        offs.append(layer * layer_bytes + tile_group_offset(dims, k) * chunk_bytes +
                    chunk_internal_offset(dims, bytes_per_px, k))
    return offs, chunk_bytes, layer_bytes
