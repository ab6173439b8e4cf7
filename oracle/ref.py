"""ctypes front-end of the REFERENCE ITSELF (test infrastructure only).

oracle/_ref/libref_downsampler.so is acquire-zarr v0.8.1's own
src/streaming/downsampler.cpp, array.dimensions.cpp, zarr.common.cpp and
src/logger/logger.cpp, compiled unmodified by `make -C oracle ref` (see the
Makefile for the recipe) and wrapped by oracle/ref_shim.cpp.  It exists only
where it was built from /root/reference (this container; the built .so
travels to the GPU box with the tree).

Only tests/, tests/golden/make_reference_vectors.py and bench.py's
cpu_baseline leg load it, as the checker or the timed CPU baseline.  The
product (acquire-zarr_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_ref", "libref_downsampler.so")
REFERENCE = "/root/reference"

NP_DTYPES = [np.uint8, np.uint16, np.uint32, np.uint64, np.int8, np.int16,
             np.int32, np.int64, np.float32, np.float64]
DTYPE_BY_NAME = {np.dtype(t).name: i for i, t in enumerate(NP_DTYPES)}


class Dim(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32),
                ("array_size_px", ctypes.c_uint32),
                ("chunk_size_px", ctypes.c_uint32),
                ("shard_size_chunks", ctypes.c_uint32),
                ("scale", ctypes.c_double)]


def build() -> str | None:
    """`make -C oracle ref` when the reference tree is present; returns the
    library path, or None when neither a build nor the tree exists."""
    if os.path.exists(os.path.join(REFERENCE, "src", "streaming", "downsampler.cpp")):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)
    return LIB_PATH if os.path.exists(LIB_PATH) else None


def available() -> bool:
    return os.path.exists(LIB_PATH)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not available():
            raise FileNotFoundError(f"{LIB_PATH} not built (make -C oracle ref)")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, u32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64
        cp = ctypes.c_char_p
        L.ref_ds_create.restype = vp
        L.ref_ds_create.argtypes = [ctypes.POINTER(Dim), u32, ctypes.c_int, ctypes.c_int, u32,
                                    cp, sz]
        L.ref_ds_destroy.argtypes = [vp]
        L.ref_ds_n_levels.argtypes = [vp]
        L.ref_ds_n_levels.restype = u32
        L.ref_ds_level_dims.argtypes = [vp, u32, ctypes.POINTER(Dim), u32]
        L.ref_ds_frame_buffer.argtypes = [vp, sz]
        L.ref_ds_frame_buffer.restype = vp
        L.ref_ds_add_buffered.argtypes = [vp, cp, sz]
        L.ref_ds_add_frame.argtypes = [vp, vp, sz, cp, sz]
        L.ref_ds_take_frame.argtypes = [vp, ctypes.c_int, vp, sz, ctypes.POINTER(sz)]
        L.ref_ds_method_string.argtypes = [vp, cp, sz]
        L.ref_ds_method_string.restype = sz
        L.ref_ds_metadata_json.argtypes = [vp, cp, sz]
        L.ref_ds_metadata_json.restype = sz
        L.ref_chunk_lattice_index.argtypes = [ctypes.POINTER(Dim), u32, u64, u32, ctypes.c_int]
        L.ref_chunk_lattice_index.restype = u32
        L.ref_tile_group_offset.argtypes = [ctypes.POINTER(Dim), u32, u64, ctypes.c_int]
        L.ref_tile_group_offset.restype = u64
        L.ref_chunk_internal_offset.argtypes = [ctypes.POINTER(Dim), u32, u64, ctypes.c_int]
        L.ref_chunk_internal_offset.restype = u64
        _lib = L
    return _lib


def _dims(dims):
    return (Dim * len(dims))(*[Dim(d[0], d[1], d[2], d[3], d[4] if len(d) > 4 else 1.0)
                               for d in dims])


class ReferenceError_(RuntimeError):
    """An exception the reference threw (message preserved)."""


class RefDownsampler:
    """zarr::Downsampler (downsampler.hh:11-64) of the reference itself.

    `dims` are (type, array_size, chunk_size, shard_size[, scale]) tuples in
    storage order, as the caller's ArrayDimensions holds them."""

    def __init__(self, dims, dtype, method, max_levels: int = 0):
        self.dtype = np.dtype(dtype)
        err = ctypes.create_string_buffer(512)
        self._h = lib().ref_ds_create(_dims(dims), len(dims), DTYPE_BY_NAME[self.dtype.name],
                                      method, max_levels, err, len(err))
        if not self._h:
            raise ReferenceError_(err.value.decode())
        self.ndims = len(dims)
        self.levels = [self.level_dims(L) for L in range(self.n_levels)]
        # (width, height, planes) per level, as add_frame reads them
        self.geometry = [(lv[-1][1], lv[-2][1], lv[-3][1]) for lv in self.levels]

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().ref_ds_destroy(h)
            self._h = None

    @property
    def n_levels(self) -> int:
        return int(lib().ref_ds_n_levels(self._h))

    def level_dims(self, level: int):
        out = (Dim * self.ndims)()
        n = lib().ref_ds_level_dims(self._h, level, out, self.ndims)
        if n < 0:
            raise KeyError(level)
        return [(o.type, o.array_size_px, o.chunk_size_px, o.shard_size_chunks, o.scale)
                for o in out[:n]]

    def add_frame(self, frame) -> None:
        buf = np.ascontiguousarray(frame).view(np.uint8).reshape(-1)
        err = ctypes.create_string_buffer(512)
        if lib().ref_ds_add_frame(self._h, buf.ctypes.data, buf.size, err, len(err)):
            raise ReferenceError_(err.value.decode())

    def load_frame(self, frame) -> None:
        """Fill the handle-owned input vector once (for timing add_buffered)."""
        buf = np.ascontiguousarray(frame).view(np.uint8).reshape(-1)
        p = lib().ref_ds_frame_buffer(self._h, buf.size)
        ctypes.memmove(p, buf.ctypes.data, buf.size)

    def add_buffered(self) -> None:
        err = ctypes.create_string_buffer(512)
        if lib().ref_ds_add_buffered(self._h, err, len(err)):
            raise ReferenceError_(err.value.decode())

    def take_frame(self, level: int):
        w, h, _ = self.geometry[level]
        out = np.empty((h, w), dtype=self.dtype)
        nb = ctypes.c_size_t(0)
        got = lib().ref_ds_take_frame(self._h, level, out.ctypes.data, out.nbytes,
                                      ctypes.byref(nb))
        if not got:
            return None
        assert nb.value == out.nbytes, (nb.value, out.nbytes)
        return out

    def take_bytes(self, level: int):
        """take_frame into a buffer sized by the reference (raw bytes)."""
        nb = ctypes.c_size_t(0)
        w, h, _ = self.geometry[level]
        out = np.empty(w * h * self.dtype.itemsize + 64, np.uint8)
        got = lib().ref_ds_take_frame(self._h, level, out.ctypes.data, out.size,
                                      ctypes.byref(nb))
        return out[:nb.value].copy() if got else None

    def downsampling_method(self) -> str:
        buf = ctypes.create_string_buffer(64)
        lib().ref_ds_method_string(self._h, buf, len(buf))
        return buf.value.decode()

    def metadata_json(self) -> str:
        n = lib().ref_ds_metadata_json(self._h, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        lib().ref_ds_metadata_json(self._h, buf, len(buf))
        return buf.value.decode()


def chunk_lattice_index(dims, frame_id: int, dim_index: int, dtype=np.uint8) -> int:
    r = lib().ref_chunk_lattice_index(_dims(dims), len(dims), frame_id, dim_index,
                                      DTYPE_BY_NAME[np.dtype(dtype).name])
    if r == 0xFFFFFFFF:
        raise ValueError("invalid dimension index")
    return int(r)


def tile_group_offset(dims, frame_id: int, dtype=np.uint8) -> int:
    return int(lib().ref_tile_group_offset(_dims(dims), len(dims), frame_id,
                                           DTYPE_BY_NAME[np.dtype(dtype).name]))


def chunk_internal_offset(dims, frame_id: int, dtype=np.uint8) -> int:
    return int(lib().ref_chunk_internal_offset(_dims(dims), len(dims), frame_id,
                                               DTYPE_BY_NAME[np.dtype(dtype).name]))
