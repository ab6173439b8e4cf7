"""CHECKER (test infrastructure only): c-blosc 1.x itself, as the image ships it.

The reference's chunk compression is `blosc_compress_ctx(clevel, shuffle,
typesize, nbytes, src, dest, nbytes + BLOSC_MAX_OVERHEAD, cname, 0, 1)`
(zarr.common.cpp:106-137; vcpkg pins `blosc >= 1.21.5`).  The library is not
in /root/reference, but this image (and the GPU box, same image) carries
c-blosc 1.21.0 at /opt/conda/lib/libblosc.so.1, linked against the liblz4
and libzstd next to it.  Loaded here through ctypes only as the checker for
aqz_blosc_* (tests/, never the product): frames the product writes must
equal the ones this library writes, byte for byte, and the filtered blocks
must equal the raw splits c-blosc stores for incompressible data.
"""
import ctypes
import os
import struct

import numpy as np

LIB_PATH = os.environ.get("AQZ_LIBBLOSC", "/opt/conda/lib/libblosc.so.1")
_lib = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(LIB_PATH)
        L.blosc_compress_ctx.restype = ctypes.c_int
        L.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                         ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                         ctypes.c_int]
        L.blosc_decompress_ctx.restype = ctypes.c_int
        L.blosc_decompress_ctx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_int]
        L.blosc_get_version_string.restype = ctypes.c_char_p
        _lib = L
    return _lib


def version() -> str:
    return lib().blosc_get_version_string().decode()


def compress(data, clevel: int, shuffle: int, typesize: int, cname: str,
             destsize: int = -1):
    """blosc_compress_ctx exactly as compress_in_place calls it (destsize
    defaults to nbytes + 16).  Returns the frame bytes, or the int status
    when it is <= 0."""
    src = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    cap = src.size + 16 if destsize < 0 else destsize
    dst = np.zeros(max(cap, 1), np.uint8)
    n = lib().blosc_compress_ctx(clevel, shuffle, typesize, src.size, src.ctypes.data,
                                 dst.ctypes.data, cap, cname.encode(), 0, 1)
    return dst[:n].tobytes() if n > 0 else n


def decompress(frame: bytes, nbytes: int) -> np.ndarray:
    src = np.frombuffer(frame, np.uint8)
    out = np.zeros(nbytes, np.uint8)
    n = lib().blosc_decompress_ctx(src.ctypes.data, out.ctypes.data, nbytes, 1)
    assert n == nbytes, n
    return out


def header(frame: bytes) -> dict:
    nbytes, blocksize, cbytes = struct.unpack_from("<III", frame, 4)
    return {"version": frame[0], "versionlz": frame[1], "flags": frame[2],
            "typesize": frame[3], "nbytes": nbytes, "blocksize": blocksize,
            "cbytes": cbytes}


def stored_splits(frame: bytes):
    """Per block, the list of (csize, payload) splits of a non-memcpyed frame."""
    h = header(frame)
    assert not h["flags"] & 0x2
    nb = -(-h["nbytes"] // h["blocksize"])
    starts = struct.unpack_from(f"<{nb}i", frame, 16)
    ends = list(starts[1:]) + [h["cbytes"]]
    blocks = []
    for s, e in zip(starts, ends):
        splits, p = [], s
        while p < e:
            (c,) = struct.unpack_from("<i", frame, p)
            splits.append((c, frame[p + 4:p + 4 + c]))
            p += 4 + c
        blocks.append(splits)
    return blocks
