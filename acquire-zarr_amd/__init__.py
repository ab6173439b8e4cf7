"""acquire-zarr MI355X multiscale downsampler — Python binding of the C ABI.

The product is the native library ``libaqz_downsampler.so`` (HIP kernels for
gfx950 + the C ABI declared in ``include/aqz_downsampler.h`` + the C++
``aqz::Downsampler`` mirror of the reference's ``zarr::Downsampler``).  This
module is a thin ctypes binding used by the tests and ``bench.py``; it never
computes anything itself and raises if the native library is missing — there
is no CPU fallback.

Import it as ``acquire_zarr_amd`` (see ``aqz_pkg.py`` at the repo root; the
directory name carries a hyphen).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# $AQZ_LIB_PATH: a variant build for A/B measurements (tools/, profiles/);
# unset, the in-tree library is the one loaded
LIB_PATH = os.environ.get("AQZ_LIB_PATH") or os.path.join(PKG_DIR, "libaqz_downsampler.so")

# ZarrDataType (zarr.types.h:55-68), ZarrDownsamplingMethod (:90-97),
# ZarrDimensionType (:81-88) numeric values.
NP_DTYPES = [np.uint8, np.uint16, np.uint32, np.uint64, np.int8, np.int16,
             np.int32, np.int64, np.float32, np.float64]
DECIMATE, MEAN, MIN, MAX = 0, 1, 2, 3
SPACE, CHANNEL, TIME, OTHER = 0, 1, 2, 3
METHODS = {"decimate": DECIMATE, "mean": MEAN, "min": MIN, "max": MAX}

# C ABI symbols (include/aqz_downsampler.h); the not-GPU test checks the
# library exports exactly these.
EXPORTS = (
    "aqz_plan_levels", "aqz_ds_create", "aqz_ds_destroy", "aqz_ds_add_frame",
    "aqz_ds_add_device_frame", "aqz_ds_take_frame", "aqz_ds_run_device_batch",
    "aqz_ds_last_batch_kind", "aqz_ds_stream_tiled_runs", "aqz_ds_run_host_batch", "aqz_ds_take_frame_tiled",
    "aqz_ds_run_device_batch_tiled", "aqz_ds_tiled_flag_slots",
    "aqz_tile_frame_device", "aqz_ds_set_level_tiling",
    "aqz_ds_add_frame_async", "aqz_ds_wait", "aqz_ds_poll", "aqz_ds_add_frame_async_take", "aqz_ds_set_input_transpose",
    "aqz_ds_take_input_frame", "aqz_transpose_frame_device",
    "aqz_blosc_filter_device", "aqz_crc32c_device", "aqz_tile_slices",
    "aqz_tile_frame_device_sliced",
    "aqz_ds_run_device_batch_chunked", "aqz_chunk_frame_offsets",
    "aqz_blosc_blocksize", "aqz_blosc_frame_from_filtered", "aqz_blosc_ctx_create",
    "aqz_blosc_ctx_destroy", "aqz_blosc_compress_device", "aqz_blosc_codec_info",
    "aqz_ds_level_bytes", "aqz_ds_level_count", "aqz_ds_device_memory_usage",
    "aqz_ds_device",
    "aqz_ds_last_error", "aqz_last_error", "aqz_method_name",
    "aqz_method_metadata_json", "aqz_version",
    "aqz_shard_unit", "aqz_node_create", "aqz_node_destroy", "aqz_node_handle_count",
    "aqz_node_handle", "aqz_node_run_host_batch", "aqz_node_last_error",
    "aqz_node_add_frame", "aqz_node_take_frame", "aqz_node_flush",
    "aqz_node_run_device_batch", "aqz_node_wait_input", "aqz_ds_wait_input",
    "aqz_node_set_level_tiling", "aqz_ds_input_pending", "aqz_node_inputs_released",
)


class AqzError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{message} (status {status})")
        self.status = status


class Dimension(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32),
                ("array_size_px", ctypes.c_uint32),
                ("chunk_size_px", ctypes.c_uint32),
                ("shard_size_chunks", ctypes.c_uint32),
                ("scale", ctypes.c_double)]


class LevelDesc(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32),
                ("height", ctypes.c_uint32),
                ("planes", ctypes.c_uint32)]


TAKE_NONE, TAKE_INTO, TAKE_HOLD = 0, 1, 2


class LevelTake(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("tile_rows", ctypes.c_uint32),
                ("tile_cols", ctypes.c_uint32), ("dst", ctypes.c_void_p),
                ("cap", ctypes.c_size_t), ("tile_nonzero", ctypes.c_void_p),
                ("nbytes", ctypes.c_size_t), ("has_frame", ctypes.c_int)]


class ChunkLattice(ctypes.Structure):
    """aqz_chunk_lattice (include/aqz_downsampler.h)."""
    _fields_ = [("device_base", ctypes.c_void_p),
                ("capacity_bytes", ctypes.c_size_t),
                ("tile_rows", ctypes.c_uint32),
                ("tile_cols", ctypes.c_uint32),
                ("chunk_stride_bytes", ctypes.c_size_t),
                ("frame_offset_bytes", ctypes.POINTER(ctypes.c_uint64))]


def chunk_frame_offsets(dims, bytes_per_px: int, first_frame: int, n_frames: int):
    """aqz_chunk_frame_offsets: (offsets[n_frames], chunk_bytes, layer_bytes)
    for storage-order `dims` = [(type, array_size, chunk_size, shard), ...]."""
    arr = (Dimension * len(dims))(*[Dimension(t, a, c, s, 1.0) for t, a, c, s in dims])
    offs = (ctypes.c_uint64 * max(n_frames, 1))()
    cb, lb = ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib().aqz_chunk_frame_offsets(arr, len(dims), bytes_per_px, first_frame, n_frames,
                                       offs, ctypes.byref(cb), ctypes.byref(lb))
    if rc:
        raise AqzError(rc, lib().aqz_last_error().decode())
    return list(offs)[:n_frames], cb.value, lb.value


_lib = None


def lib() -> ctypes.CDLL:
    """Load the native library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C acquire-zarr_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
    L.aqz_plan_levels.argtypes = [ctypes.POINTER(Dimension), u32, u32,
                                  ctypes.POINTER(Dimension), u32, ctypes.POINTER(u32)]
    L.aqz_ds_create.argtypes = [ctypes.POINTER(LevelDesc), u32, i32, i32, i32,
                                ctypes.POINTER(vp)]
    L.aqz_ds_destroy.argtypes = [vp]
    L.aqz_ds_destroy.restype = None
    L.aqz_ds_add_frame.argtypes = [vp, vp, sz]
    L.aqz_ds_add_frame_async.argtypes = [vp, vp, sz]
    L.aqz_ds_add_frame_async_take.argtypes = [vp, vp, sz, ctypes.POINTER(LevelTake)]
    L.aqz_ds_wait.argtypes = [vp]
    L.aqz_ds_poll.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.aqz_ds_set_input_transpose.argtypes = [vp, ctypes.c_int]
    L.aqz_ds_take_input_frame.argtypes = [vp, u32, u32, vp, sz, vp, ctypes.POINTER(sz),
                                          ctypes.POINTER(ctypes.c_int)]
    L.aqz_transpose_frame_device.argtypes = [ctypes.c_int, vp, u32, u32, vp, vp]
    L.aqz_tile_slices.argtypes = [u32, u32]
    L.aqz_tile_slices.restype = u32
    L.aqz_tile_frame_device_sliced.argtypes = [i32, vp, u32, u32, u32, u32, vp, vp, vp]
    L.aqz_blosc_filter_device.argtypes = [ctypes.c_int, u32, u32, vp, sz, u32, vp, vp]
    L.aqz_crc32c_device.argtypes = [vp, sz, sz, u32, vp, vp]
    L.aqz_blosc_blocksize.argtypes = [ctypes.c_int, u32, sz, ctypes.c_char_p,
                                      ctypes.POINTER(u32)]
    L.aqz_blosc_frame_from_filtered.argtypes = [ctypes.c_int, ctypes.c_int, u32,
                                                ctypes.c_char_p, vp, vp, sz, vp, sz,
                                                ctypes.POINTER(sz), ctypes.POINTER(ctypes.c_int)]
    L.aqz_blosc_ctx_create.argtypes = [i32, u32, ctypes.POINTER(vp)]
    L.aqz_blosc_ctx_destroy.argtypes = [vp]
    L.aqz_blosc_ctx_destroy.restype = None
    L.aqz_blosc_compress_device.argtypes = [vp, ctypes.c_int, ctypes.c_int, u32,
                                            ctypes.c_char_p, vp, sz, u32, vp, sz,
                                            ctypes.POINTER(sz), vp]
    L.aqz_blosc_codec_info.argtypes = []
    L.aqz_blosc_codec_info.restype = ctypes.c_char_p
    L.aqz_ds_add_device_frame.argtypes = [vp, vp, sz]
    L.aqz_ds_take_frame.argtypes = [vp, u32, vp, sz, ctypes.POINTER(sz),
                                    ctypes.POINTER(i32)]
    L.aqz_ds_run_device_batch.argtypes = [vp, vp, u32, ctypes.POINTER(vp),
                                          ctypes.POINTER(u32), vp]
    L.aqz_ds_run_device_batch_tiled.argtypes = [vp, vp, u32, ctypes.POINTER(u32),
                                                ctypes.POINTER(u32), ctypes.POINTER(vp),
                                                ctypes.POINTER(vp), ctypes.POINTER(u32), vp]
    L.aqz_ds_run_device_batch_chunked.argtypes = [vp, vp, u32, ctypes.POINTER(ChunkLattice),
                                                  ctypes.POINTER(vp), ctypes.POINTER(u32), vp]
    L.aqz_chunk_frame_offsets.argtypes = [ctypes.POINTER(Dimension), u32, u32, ctypes.c_uint64,
                                          u32, ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_uint64)]
    L.aqz_ds_tiled_flag_slots.argtypes = [vp, u32, u32, u32]
    L.aqz_ds_tiled_flag_slots.restype = u32
    L.aqz_ds_take_frame_tiled.argtypes = [vp, u32, u32, u32, vp, sz, vp,
                                          ctypes.POINTER(sz), ctypes.POINTER(i32)]
    L.aqz_ds_set_level_tiling.argtypes = [vp, u32, u32, u32]
    L.aqz_tile_frame_device.argtypes = [i32, vp, u32, u32, u32, u32, vp, vp, vp]
    L.aqz_ds_run_host_batch.argtypes = [vp, vp, u32, ctypes.POINTER(vp),
                                        ctypes.POINTER(u32)]
    L.aqz_ds_last_batch_kind.argtypes = [vp]
    L.aqz_ds_last_batch_kind.restype = i32
    L.aqz_ds_stream_tiled_runs.argtypes = [vp]
    L.aqz_ds_stream_tiled_runs.restype = ctypes.c_uint64
    L.aqz_ds_level_bytes.argtypes = [vp, u32]
    L.aqz_ds_level_bytes.restype = sz
    L.aqz_ds_level_count.argtypes = [vp]
    L.aqz_ds_level_count.restype = u32
    L.aqz_ds_device_memory_usage.argtypes = [vp]
    L.aqz_ds_device_memory_usage.restype = sz
    L.aqz_ds_device.argtypes = [vp]
    L.aqz_ds_device.restype = i32
    L.aqz_ds_last_error.argtypes = [vp]
    L.aqz_ds_last_error.restype = ctypes.c_char_p
    L.aqz_last_error.argtypes = []
    L.aqz_last_error.restype = ctypes.c_char_p
    L.aqz_method_name.argtypes = [i32]
    L.aqz_method_name.restype = ctypes.c_char_p
    L.aqz_method_metadata_json.argtypes = [i32]
    L.aqz_method_metadata_json.restype = ctypes.c_char_p
    L.aqz_version.argtypes = []
    L.aqz_version.restype = ctypes.c_char_p
    L.aqz_shard_unit.argtypes = [ctypes.POINTER(LevelDesc), u32, ctypes.POINTER(u32),
                                 ctypes.POINTER(u32)]
    L.aqz_node_create.argtypes = [ctypes.POINTER(LevelDesc), u32, i32, i32,
                                  ctypes.POINTER(i32), u32, ctypes.POINTER(vp)]
    L.aqz_node_destroy.argtypes = [vp]
    L.aqz_node_destroy.restype = None
    L.aqz_node_handle_count.argtypes = [vp]
    L.aqz_node_handle_count.restype = u32
    L.aqz_node_handle.argtypes = [vp, u32]
    L.aqz_node_handle.restype = vp
    L.aqz_node_run_host_batch.argtypes = [vp, vp, u32, ctypes.POINTER(vp), ctypes.POINTER(u32)]
    L.aqz_node_last_error.argtypes = [vp]
    L.aqz_node_last_error.restype = ctypes.c_char_p
    L.aqz_node_add_frame.argtypes = [vp, vp, sz]
    L.aqz_node_take_frame.argtypes = [vp, u32, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(i32)]
    L.aqz_node_flush.argtypes = [vp]
    L.aqz_node_wait_input.argtypes = [vp]
    L.aqz_node_set_level_tiling.argtypes = [vp, u32, u32, u32]
    L.aqz_ds_wait_input.argtypes = [vp]
    L.aqz_ds_input_pending.argtypes = [vp, ctypes.POINTER(i32)]
    L.aqz_node_inputs_released.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    L.aqz_node_run_device_batch.argtypes = [vp, vp, i32, u32, ctypes.POINTER(vp),
                                            ctypes.POINTER(u32), vp, u32]
    _lib = L
    return L


def dtype_code(dt) -> int:
    name = np.dtype(dt).name
    for i, t in enumerate(NP_DTYPES):
        if np.dtype(t).name == name:
            return i
    raise ValueError(f"unsupported dtype {dt}")


def plan_levels(dims, max_levels: int = 0):
    """Level planner (make_writer_configurations_, downsampler.cpp:493-597).

    `dims`: storage-order (type, size, chunk, shard[, scale]) tuples; a 2-D
    list gets the reference's phantom singleton dimension prepended
    (array.dimensions.cpp:149-152).  Returns one list of tuples per level.
    """
    dims = list(dims)
    if len(dims) == 2:
        dims = [(OTHER, 1, 1, 1, 1.0)] + dims
    nd = len(dims)
    arr = (Dimension * nd)(*[Dimension(d[0], d[1], d[2], d[3],
                                       d[4] if len(d) > 4 else 1.0) for d in dims])
    n = ctypes.c_uint32(0)
    L = lib()
    rc = L.aqz_plan_levels(arr, nd, max_levels, None, 0, ctypes.byref(n))
    if rc:
        raise AqzError(rc, L.aqz_last_error().decode())
    out = (Dimension * (nd * n.value))()
    rc = L.aqz_plan_levels(arr, nd, max_levels, out, n.value, ctypes.byref(n))
    if rc:
        raise AqzError(rc, L.aqz_last_error().decode())
    return [[(o.type, o.array_size_px, o.chunk_size_px, o.shard_size_chunks, o.scale)
             for o in out[l * nd:(l + 1) * nd]] for l in range(n.value)]


def level_geometry(levels):
    """(width, height, planes) per level, as add_frame reads them."""
    return [(lv[-1][1], lv[-2][1], lv[-3][1]) for lv in levels]


def method_name(method: int):
    r = lib().aqz_method_name(method)
    return None if r is None else r.decode()


def method_metadata(method: int):
    import json
    r = lib().aqz_method_metadata_json(method)
    return None if r is None else json.loads(r.decode())


class Downsampler:
    """Binding of one ``aqz_ds`` handle: the GPU replacement of
    ``zarr::Downsampler`` (downsampler.hh:11-64).

    ``geometry`` is the per-level (width, height, planes) list (see
    ``level_geometry(plan_levels(...))``).
    """

    def __init__(self, geometry, dtype, method: int, device: int = -1):
        self.dtype = np.dtype(dtype)
        self.geometry = [tuple(int(x) for x in g) for g in geometry]
        n = len(self.geometry)
        desc = (LevelDesc * n)(*[LevelDesc(*g) for g in self.geometry])
        h = ctypes.c_void_p()
        L = lib()
        rc = L.aqz_ds_create(desc, n, dtype_code(self.dtype), method, device,
                             ctypes.byref(h))
        if rc:
            raise AqzError(rc, L.aqz_last_error().decode())
        self._h = h
        self.method = method
        self._pending = None  # frame of a pending add_frame_async
        self._takes = None    # (LevelTake array, buffers) of add_frame_async_take

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib().aqz_ds_destroy(h)
        self._h = None

    __del__ = close

    def _check(self, rc):
        if rc:
            raise AqzError(rc, lib().aqz_ds_last_error(self._h).decode())

    @property
    def n_levels(self) -> int:
        return len(self.geometry)

    def level_bytes(self, level: int) -> int:
        return lib().aqz_ds_level_bytes(self._h, level)

    def set_level_tiling(self, level: int, tile_rows: int, tile_cols: int):
        self._check(lib().aqz_ds_set_level_tiling(self._h, level, tile_rows, tile_cols))

    def take_frame_tiled(self, level: int, tile_rows: int, tile_cols: int):
        """Chunk-tiled take: (tiles[n_tiles, tile_rows, tile_cols],
        nonzero[n_tiles] bool) or None."""
        if not 0 <= level < self.n_levels:
            return None
        w, h, _ = self.geometry[level]
        nt = (-(-h // tile_rows)) * (-(-w // tile_cols))
        out = np.empty((nt, tile_rows, tile_cols), dtype=self.dtype)
        nz = np.empty(nt, dtype=np.uint8)
        nb, has = ctypes.c_size_t(0), ctypes.c_int(0)
        self._check(lib().aqz_ds_take_frame_tiled(
            self._h, level, tile_rows, tile_cols, out.ctypes.data, out.nbytes,
            nz.ctypes.data, ctypes.byref(nb), ctypes.byref(has)))
        return (out, nz.astype(bool)) if has.value else None

    def set_input_transpose(self, transpose: bool):
        """aqz_ds_set_input_transpose: frames arrive in acquisition order
        (levels[0].width rows x levels[0].height columns)."""
        self._check(lib().aqz_ds_set_input_transpose(self._h, 1 if transpose else 0))

    def take_input_frame(self, tile_rows: int = 0, tile_cols: int = 0):
        """Last added level-0 frame in storage order: (h, w) array when
        untiled, else (tiles, nonzero) like take_frame_tiled; None if none."""
        w, h, _ = self.geometry[0]
        nb, has = ctypes.c_size_t(0), ctypes.c_int(0)
        if tile_rows == 0 and tile_cols == 0:
            out = np.empty((h, w), dtype=self.dtype)
            self._check(lib().aqz_ds_take_input_frame(
                self._h, 0, 0, out.ctypes.data, out.nbytes, None, ctypes.byref(nb),
                ctypes.byref(has)))
            return out if has.value else None
        # a half-zero tile shape is passed through for the C ABI to reject
        nt = (-(-h // tile_rows)) * (-(-w // tile_cols)) if tile_rows and tile_cols else 1
        out = np.empty((nt, max(tile_rows, 1), max(tile_cols, 1)), dtype=self.dtype)
        nz = np.empty(nt, dtype=np.uint8)
        self._check(lib().aqz_ds_take_input_frame(
            self._h, tile_rows, tile_cols, out.ctypes.data, out.nbytes, nz.ctypes.data,
            ctypes.byref(nb), ctypes.byref(has)))
        return (out, nz.astype(bool)) if has.value else None

    def run_host_batch(self, host_frames: int, n_frames: int, host_outs):
        """Pipelined host batch: `host_frames` and `host_outs[L]` are host
        addresses (index 0 ignored).  Returns frames emitted per level."""
        n = self.n_levels
        outs = (ctypes.c_void_p * n)(*[int(p) if p else 0 for p in host_outs])
        counts = (ctypes.c_uint32 * n)()
        self._check(lib().aqz_ds_run_host_batch(self._h, host_frames, n_frames,
                                                outs, counts))
        return list(counts)

    def last_batch_kind(self) -> int:
        """0 per-frame, 1 fused 2-D cascade, 2 fused volume, 3 2-D batch with
        some runs on batched single-level kernels, 4 fused 2-D cascade writing
        chunk tiles, -1 none."""
        return lib().aqz_ds_last_batch_kind(self._h)

    def stream_tiled_runs(self) -> int:
        """Pure-XY level runs add_frame tiled in the cascade launch itself."""
        return int(lib().aqz_ds_stream_tiled_runs(self._h))

    def device_memory_usage(self) -> int:
        return lib().aqz_ds_device_memory_usage(self._h)

    def device(self) -> int:
        """HIP ordinal the handle runs on."""
        return lib().aqz_ds_device(self._h)

    def add_frame(self, frame: np.ndarray):
        frame = np.ascontiguousarray(frame)
        if frame.dtype != self.dtype:
            raise TypeError(f"frame dtype {frame.dtype} != {self.dtype}")
        self._check(lib().aqz_ds_add_frame(self._h, frame.ctypes.data, frame.nbytes))

    def add_frame_async(self, frame: np.ndarray):
        """aqz_ds_add_frame_async: returns at once; `frame` is kept alive
        (and must not be modified) until wait() or the next call."""
        frame = np.ascontiguousarray(frame)
        if frame.dtype != self.dtype:
            raise TypeError(f"frame dtype {frame.dtype} != {self.dtype}")
        # The C call first settles the previous job, whose upload may still be
        # reading the previous frame: keep that frame alive until it returns.
        prev, self._pending = self._pending, frame
        try:
            self._check(lib().aqz_ds_add_frame_async(self._h, frame.ctypes.data,
                                                     frame.nbytes))
        finally:
            del prev

    def wait(self):
        try:
            self._check(lib().aqz_ds_wait(self._h))
        finally:
            self._pending = None

    def poll(self) -> bool:
        """aqz_ds_poll: True once no add_frame_async job is running."""
        done = ctypes.c_int(0)
        self._check(lib().aqz_ds_poll(self._h, ctypes.byref(done)))
        return bool(done.value)

    def add_frame_async_take(self, frame: np.ndarray, tiles, hold=()):
        """aqz_ds_add_frame_async_take: every level L >= 1 taken in the
        background job right behind the add — chunk-tiled when tiles[L] =
        (tile_rows, tile_cols), row-major when tiles[L] is None — except the
        levels in `hold` (AQZ_TAKE_HOLD).  wait_takes() returns the results."""
        frame = np.ascontiguousarray(frame)
        if frame.dtype != self.dtype:
            raise TypeError(f"frame dtype {frame.dtype} != {self.dtype}")
        n = self.n_levels
        arr = (LevelTake * n)()
        bufs = [None] * n
        for L in range(1, n):
            w, h, _ = self.geometry[L]
            if L in hold:
                arr[L].mode = TAKE_HOLD
                continue
            t = tiles[L] if tiles is not None else None
            if t:
                tr, tc = t
                nt = (-(-h // tr)) * (-(-w // tc))
                out = np.empty((nt, tr, tc), dtype=self.dtype)
                nz = np.empty(nt, dtype=np.uint8)
                arr[L] = LevelTake(TAKE_INTO, tr, tc, out.ctypes.data, out.nbytes,
                                   nz.ctypes.data, 0, 0)
                bufs[L] = (out, nz)
            else:
                out = np.empty((h, w), dtype=self.dtype)
                arr[L] = LevelTake(TAKE_INTO, 0, 0, out.ctypes.data, out.nbytes, None, 0, 0)
                bufs[L] = (out, None)
        prev, self._pending = self._pending, frame
        try:
            self._check(lib().aqz_ds_add_frame_async_take(self._h, frame.ctypes.data,
                                                          frame.nbytes, arr))
            self._takes = (arr, bufs)
        finally:
            del prev

    def wait_takes(self):
        """Wait for add_frame_async_take; per level None (no frame, or held),
        a row-major (h, w) array, or (tiles, zero-scan bools)."""
        arr, bufs = self._takes
        try:
            self.wait()
        finally:
            self._takes = None
        out = [None] * self.n_levels
        for L in range(1, self.n_levels):
            if arr[L].mode != TAKE_INTO or not arr[L].has_frame:
                continue
            a, nz = bufs[L]
            out[L] = a if nz is None else (a, nz.astype(bool))
        return out

    def add_device_frame(self, device_ptr: int, nbytes: int):
        self._check(lib().aqz_ds_add_device_frame(self._h, device_ptr, nbytes))

    def take_frame(self, level: int):
        """Cached frame of `level` as an (h, w) array, or None."""
        w, h, _ = self.geometry[level] if 0 <= level < self.n_levels else (0, 0, 0)
        out = np.empty((max(h, 1), max(w, 1)), dtype=self.dtype)
        nb = ctypes.c_size_t(0)
        has = ctypes.c_int(0)
        self._check(lib().aqz_ds_take_frame(self._h, level, out.ctypes.data,
                                            out.nbytes, ctypes.byref(nb),
                                            ctypes.byref(has)))
        return out if has.value else None

    def run_device_batch_tiled(self, device_frames: int, n_frames: int, tiles,
                               device_outs, device_nonzero=None, stream: int = 0):
        """Device-resident batch with every level chunk-tiled by the pyramid
        kernel: `tiles[L]` = (tile_rows, tile_cols), `device_outs[L]` /
        `device_nonzero[L]` device pointers (index 0 ignored; nonzero
        optional, tiled_flag_slots(L, ...) bytes per tile).  Returns frames
        emitted per level."""
        n = self.n_levels
        tr = (ctypes.c_uint32 * n)(*[int(t[0]) if t else 0 for t in tiles])
        tc = (ctypes.c_uint32 * n)(*[int(t[1]) if t else 0 for t in tiles])
        outs = (ctypes.c_void_p * n)(*[int(p) if p else 0 for p in device_outs])
        nz = None
        if device_nonzero is not None:
            nz = (ctypes.c_void_p * n)(*[int(p) if p else 0 for p in device_nonzero])
        counts = (ctypes.c_uint32 * n)()
        self._check(lib().aqz_ds_run_device_batch_tiled(
            self._h, device_frames, n_frames, tr, tc, outs, nz, counts,
            ctypes.c_void_p(stream) if stream else None))
        return list(counts)

    def run_device_batch_chunked(self, device_frames: int, n_frames: int, lattices,
                                 device_nonzero=None, stream: int = 0):
        """aqz_ds_run_device_batch_chunked: `lattices[L]` = (device_base,
        capacity_bytes, tile_rows, tile_cols, chunk_stride_bytes,
        frame_offset_bytes list) per level (index 0 ignored)."""
        n = self.n_levels
        arr = (ChunkLattice * n)()
        keep = []
        for L in range(1, n):
            base, cap, tr, tc, stride, offs = lattices[L]
            o = (ctypes.c_uint64 * max(n_frames, 1))(*offs)
            keep.append(o)
            arr[L] = ChunkLattice(int(base), cap, tr, tc, stride, o)
        nz = None
        if device_nonzero is not None:
            nz = (ctypes.c_void_p * n)(*[int(p) if p else 0 for p in device_nonzero])
        counts = (ctypes.c_uint32 * n)()
        self._check(lib().aqz_ds_run_device_batch_chunked(
            self._h, device_frames, n_frames, arr, nz, counts,
            ctypes.c_void_p(stream) if stream else None))
        return list(counts)

    def batch_call(self, device_frames: int, n_frames: int, device_outs, stream: int = 0,
                   tiles=None, device_nonzero=None):
        """A prepared aqz_ds_run_device_batch (or, with `tiles`,
        aqz_ds_run_device_batch_tiled) call: the ctypes argument arrays are
        built once, so each call costs one foreign call — what a benchmark
        loop of short launches needs to keep the stream fed.  Returns a
        function that runs one batch and returns the per-level counts."""
        n = self.n_levels
        L = lib()
        outs = (ctypes.c_void_p * n)(*[int(p) if p else 0 for p in device_outs])
        counts = (ctypes.c_uint32 * n)()
        st = ctypes.c_void_p(stream) if stream else None
        h = self._h
        if tiles is None:
            fn, args = L.aqz_ds_run_device_batch, (h, device_frames, n_frames, outs, counts, st)
        else:
            tr = (ctypes.c_uint32 * n)(*[int(t[0]) if t else 0 for t in tiles])
            tc = (ctypes.c_uint32 * n)(*[int(t[1]) if t else 0 for t in tiles])
            nz = None
            if device_nonzero is not None:
                nz = (ctypes.c_void_p * n)(*[int(p) if p else 0 for p in device_nonzero])
            fn = L.aqz_ds_run_device_batch_tiled
            args = (h, device_frames, n_frames, tr, tc, outs, nz, counts, st)

        def call():
            rc = fn(*args)
            if rc:
                self._check(rc)
            return counts
        return call

    def tiled_flag_slots(self, level: int, tile_rows: int, tile_cols: int) -> int:
        """Zero-scan flag bytes per tile of run_device_batch_tiled at `level`."""
        return lib().aqz_ds_tiled_flag_slots(self._h, level, tile_rows, tile_cols)

    def run_device_batch(self, device_frames: int, n_frames: int, device_outs,
                         stream: int = 0):
        """Device-resident batch: `device_outs[L]` are device pointers
        (index 0 ignored).  Returns frames emitted per level."""
        n = self.n_levels
        outs = (ctypes.c_void_p * n)(*[int(p) if p else 0 for p in device_outs])
        counts = (ctypes.c_uint32 * n)()
        self._check(lib().aqz_ds_run_device_batch(
            self._h, device_frames, n_frames, outs, counts,
            ctypes.c_void_p(stream) if stream else None))
        return list(counts)


def tile_frame_device(dtype, device_frame: int, width: int, height: int,
                      tile_rows: int, tile_cols: int, device_tiles: int,
                      device_nonzero: int, stream: int = 0):
    """aqz_tile_frame_device (asynchronous on `stream`)."""
    L = lib()
    rc = L.aqz_tile_frame_device(dtype_code(dtype), device_frame, width, height,
                                 tile_rows, tile_cols, device_tiles, device_nonzero,
                                 ctypes.c_void_p(stream) if stream else None)
    if rc:
        raise AqzError(rc, L.aqz_last_error().decode())


def tile_slices(tile_rows: int, tile_cols: int) -> int:
    return lib().aqz_tile_slices(tile_rows, tile_cols)


def tile_frame_device_sliced(dtype, device_frame: int, width: int, height: int,
                             tile_rows: int, tile_cols: int, device_tiles: int,
                             device_slice_flags: int, stream: int = 0):
    """aqz_tile_frame_device_sliced (asynchronous on `stream`)."""
    L = lib()
    rc = L.aqz_tile_frame_device_sliced(dtype_code(dtype), device_frame, width, height,
                                        tile_rows, tile_cols, device_tiles,
                                        device_slice_flags,
                                        ctypes.c_void_p(stream) if stream else None)
    if rc:
        raise AqzError(rc, L.aqz_last_error().decode())


def transpose_frame_device(dtype, device_src: int, rows: int, cols: int,
                           device_dst: int, stream: int = 0):
    """aqz_transpose_frame_device (asynchronous on `stream`)."""
    L = lib()
    rc = L.aqz_transpose_frame_device(dtype_code(dtype), device_src, rows, cols,
                                      device_dst,
                                      ctypes.c_void_p(stream) if stream else None)
    if rc:
        raise AqzError(rc, L.aqz_last_error().decode())


NOSHUFFLE, SHUFFLE, BITSHUFFLE = 0, 1, 2  # aqz_codec.h


def blosc_filter_device(shuffle: int, typesize: int, blocksize: int, device_src: int,
                        nbytes: int, n_buffers: int, device_dst: int, stream: int = 0):
    """aqz_blosc_filter_device (asynchronous on `stream`)."""
    L = lib()
    rc = L.aqz_blosc_filter_device(shuffle, typesize, blocksize, device_src, nbytes,
                                   n_buffers, device_dst,
                                   ctypes.c_void_p(stream) if stream else None)
    if rc:
        raise AqzError(rc, L.aqz_last_error().decode())


BLOSC_MAX_OVERHEAD = 16  # aqz_blosc.h


def _raise_if(rc):
    if rc:
        raise AqzError(rc, lib().aqz_last_error().decode())


def blosc_blocksize(clevel: int, typesize: int, nbytes: int, cname: str) -> int:
    """aqz_blosc_blocksize: c-blosc's compute_blocksize for blosc_compress_ctx."""
    bs = ctypes.c_uint32()
    _raise_if(lib().aqz_blosc_blocksize(clevel, typesize, nbytes, cname.encode(),
                                        ctypes.byref(bs)))
    return bs.value


def blosc_frame_from_filtered(clevel: int, shuffle: int, typesize: int, cname: str,
                              filtered, src=None, destsize: int = -1):
    """aqz_blosc_frame_from_filtered on host arrays.  Returns (frame bytes,
    raw_needed); with `src` None and raw_needed set, the frame still lacks
    the raw chunk after its 16-byte header."""
    f = np.ascontiguousarray(filtered).view(np.uint8).reshape(-1)
    s = None if src is None else np.ascontiguousarray(src).view(np.uint8).reshape(-1)
    n = f.size
    cap = n + BLOSC_MAX_OVERHEAD if destsize < 0 else destsize
    dest = np.zeros(max(cap, 1), np.uint8)
    out, raw = ctypes.c_size_t(), ctypes.c_int()
    _raise_if(lib().aqz_blosc_frame_from_filtered(
        clevel, shuffle, typesize, cname.encode(), f.ctypes.data,
        None if s is None else s.ctypes.data, n, dest.ctypes.data, cap,
        ctypes.byref(out), ctypes.byref(raw)))
    return dest[:out.value].tobytes(), bool(raw.value)


class BloscContext:
    """aqz_blosc_ctx: compress_in_place (zarr.common.cpp:106-137) for many
    device chunk buffers at once."""

    def __init__(self, device: int = 0, n_threads: int = 0):
        h = ctypes.c_void_p()
        _raise_if(lib().aqz_blosc_ctx_create(device, n_threads, ctypes.byref(h)))
        self._h = h

    def close(self):
        if self._h:
            lib().aqz_blosc_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compress_device(self, clevel: int, shuffle: int, typesize: int, cname: str,
                        device_src: int, nbytes: int, n_buffers: int, stream: int = 0,
                        host_dst=None, dst_stride: int = 0):
        """Frames of `n_buffers` device chunks of `nbytes`; returns the list of
        frames (bytes) when `host_dst` is None, else the frame sizes."""
        stride = dst_stride or nbytes + BLOSC_MAX_OVERHEAD
        own = host_dst is None
        if own:
            host_dst = np.empty(n_buffers * stride, np.uint8)
        sizes = (ctypes.c_size_t * n_buffers)()
        _raise_if(lib().aqz_blosc_compress_device(
            self._h, clevel, shuffle, typesize, cname.encode(), device_src, nbytes,
            n_buffers, host_dst.ctypes.data, stride, sizes,
            ctypes.c_void_p(stream) if stream else None))
        if not own:
            return list(sizes)
        return [host_dst[k * stride:k * stride + sizes[k]].tobytes() for k in range(n_buffers)]


def blosc_codec_info() -> str:
    return lib().aqz_blosc_codec_info().decode()


def crc32c_device(device_data: int, nbytes: int, stride: int, n_buffers: int,
                  device_crcs: int, stream: int = 0):
    """aqz_crc32c_device (asynchronous on `stream`)."""
    L = lib()
    rc = L.aqz_crc32c_device(device_data, nbytes, stride, n_buffers, device_crcs,
                             ctypes.c_void_p(stream) if stream else None)
    if rc:
        raise AqzError(rc, L.aqz_last_error().decode())


def alg_bytes_per_frame(geometry, bpp: int) -> int:
    """Algorithmic HBM bytes per 2-D frame: read level 0 once, write every
    output level once."""
    w0, h0, _ = geometry[0]
    total = w0 * h0 * bpp
    for w, h, _ in geometry[1:]:
        total += w * h * bpp
    return total


def shard_unit(geometry):
    """(unit, frames emitted per level per unit) of a pyramid (aqz_shard_unit):
    the slab of level-0 frames a node deals to one GPU at a time."""
    n = len(geometry)
    desc = (LevelDesc * n)(*[LevelDesc(*g) for g in geometry])
    u = ctypes.c_uint32(0)
    per = (ctypes.c_uint32 * n)()
    L = lib()
    rc = L.aqz_shard_unit(desc, n, ctypes.byref(u), per)
    if rc:
        raise AqzError(rc, L.aqz_last_error().decode())
    return u.value, list(per)


class Node:
    """Binding of an ``aqz_node``: frames sharded over `devices` (SURVEY
    §8(e)); run_host_batch returns each level in frame-id order."""

    def __init__(self, geometry, dtype, method: int, devices):
        self.dtype = np.dtype(dtype)
        self.geometry = [tuple(int(x) for x in g) for g in geometry]
        n = len(self.geometry)
        desc = (LevelDesc * n)(*[LevelDesc(*g) for g in self.geometry])
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        L = lib()
        rc = L.aqz_node_create(desc, n, dtype_code(self.dtype), method, devs, len(devices),
                               ctypes.byref(h))
        if rc:
            raise AqzError(rc, L.aqz_last_error().decode())
        self._h = h
        self.unit, self.frames_per_unit = shard_unit(self.geometry)
        # frames handed to aqz_node_add_frame stay referenced until their
        # handle is reused (unit x handles adds later) or flush() returns
        import collections
        self._inflight = collections.deque(maxlen=self.unit * len(devices) + 1)

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            lib().aqz_node_destroy(h)
            self._h = None
        if hasattr(self, "_inflight"):
            self._inflight.clear()

    def _check(self, rc):
        if rc:
            raise AqzError(rc, lib().aqz_node_last_error(self._h).decode())

    def add_frame(self, frame: np.ndarray):
        """aqz_node_add_frame: deal the frame to its handle, return at once."""
        frame = np.ascontiguousarray(frame)
        if frame.dtype != self.dtype:
            raise TypeError(f"frame dtype {frame.dtype} != {self.dtype}")
        self._check(lib().aqz_node_add_frame(self._h, frame.ctypes.data, frame.nbytes))
        self._inflight.append(frame)

    def take_frame(self, level: int):
        """Next level frame in emission order, or None if none is ready."""
        w, h, _ = self.geometry[level]
        out = np.empty((h, w), dtype=self.dtype)
        nb = ctypes.c_size_t(0)
        has = ctypes.c_int(0)
        self._check(lib().aqz_node_take_frame(self._h, level, out.ctypes.data, out.nbytes,
                                              ctypes.byref(nb), ctypes.byref(has)))
        return out if has.value else None

    def flush(self):
        try:
            self._check(lib().aqz_node_flush(self._h))
        finally:
            self._inflight.clear()

    def wait_input(self):
        """aqz_node_wait_input: every frame added so far is uploaded (the
        caller may reuse its buffers); their levels may still be running."""
        self._check(lib().aqz_node_wait_input(self._h))
        self._inflight.clear()

    def inputs_released(self) -> int:
        """aqz_node_inputs_released: how many of the frames added so far (a
        prefix, in add order) no upload still reads — non-blocking."""
        r = ctypes.c_uint64(0)
        self._check(lib().aqz_node_inputs_released(self._h, ctypes.byref(r)))
        return r.value

    def __del__(self):
        self.close()

    def handle_devices(self):
        L = lib()
        return [L.aqz_ds_device(L.aqz_node_handle(self._h, i))
                for i in range(L.aqz_node_handle_count(self._h))]

    def run_host_batch(self, host_frames: int, n_frames: int, host_outs):
        """host_frames / host_outs[L] are host addresses (index 0 ignored)."""
        n = len(self.geometry)
        outs = (ctypes.c_void_p * n)(*([None] + [int(p) for p in host_outs[1:]]))
        counts = (ctypes.c_uint32 * n)()
        L = lib()
        rc = L.aqz_node_run_host_batch(self._h, host_frames, n_frames, outs, counts)
        if rc:
            raise AqzError(rc, L.aqz_node_last_error(self._h).decode())
        return list(counts)

    def device_batch_call(self, device_frames: int, src_device: int, n_frames: int,
                          device_outs, stream: int = 0, stage_all: bool = False):
        """A prepared aqz_node_run_device_batch: device addresses on
        `src_device` (device_outs index 0 ignored); the returned callable
        launches once per call and returns the per-level counts."""
        n = len(self.geometry)
        outs = (ctypes.c_void_p * n)(*([None] + [int(p) for p in device_outs[1:]]))
        counts = (ctypes.c_uint32 * n)()
        L = lib()
        fn = L.aqz_node_run_device_batch
        flags = 1 if stage_all else 0  # AQZ_NODE_STAGE_ALL
        args = (self._h, ctypes.c_void_p(device_frames), src_device, n_frames, outs, counts,
                ctypes.c_void_p(stream or None), flags)

        def call():
            rc = fn(*args)
            if rc:
                raise AqzError(rc, L.aqz_node_last_error(self._h).decode())
            return list(counts)
        return call

    def run_device_batch(self, device_frames: int, src_device: int, n_frames: int,
                         device_outs, stream: int = 0, stage_all: bool = False):
        """aqz_node_run_device_batch (asynchronous on `stream`)."""
        return self.device_batch_call(device_frames, src_device, n_frames, device_outs,
                                      stream, stage_all)()
