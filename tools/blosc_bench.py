"""Chunk compression of one headline frame's level-0 chunks (256 chunks of
256x256 u16 = 128 KiB): compress_in_place (zarr.common.cpp:106-137) per chunk.

  cblosc   : the image's c-blosc 1.21.0, blosc_compress_ctx(nthreads=1) per
             chunk, chunks spread over T pthreads (oracle/blosc_cpu.c; the
             reference runs one compression job per chunk on its thread
             pool) — host-resident input, no Python in the loop;
  aqz      : aqz_blosc_compress_device on the device-resident chunks: GPU
             filter, grouped D2H of the filtered chunks, LZ4/zstd on T host
             threads — device-resident input (the chunks the tiled pyramid or
             tile kernel leave in HBM), host frames out.
Frames are checked equal before timing.  Prints one JSON line per case.

Run: python tools/blosc_bench.py [--threads 16] [--reps 5]
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]


def chunks_u16(n, rng):
    yy, xx = np.mgrid[0:256, 0:256]
    out = np.empty((n, 256, 256), np.uint16)
    for k in range(n):
        base = 2000 + 500 * np.sin((xx + 13 * k) / 17.0) * np.cos((yy - 5 * k) / 23.0)
        out[k] = (base + rng.normal(0, 4, (256, 256))).astype(np.uint16)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--chunks", type=int, default=256)
    a = p.parse_args()
    import torch
    import aqz_pkg
    import blosc_ref
    aqz = aqz_pkg.load()
    rng = np.random.default_rng(1)
    host = chunks_u16(a.chunks, rng)
    raw = host.view(np.uint8).reshape(-1)
    nb = 256 * 256 * 2
    d = torch.from_numpy(raw.copy()).to("cuda")
    torch.cuda.synchronize()
    ctx = aqz.BloscContext(0, a.threads)
    stride = nb + 16
    dst = np.empty(a.chunks * stride, np.uint8)
    pool = ThreadPoolExecutor(a.threads)
    import ctypes
    cpu = ctypes.CDLL(os.path.join(ROOT, "oracle", "libblosc_cpu.so"))
    cpu.cblosc_compress_chunks.restype = ctypes.c_double
    cpu.cblosc_compress_chunks.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
    cdst = np.empty(a.chunks * (nb + 16), np.uint8)
    csizes = (ctypes.c_size_t * a.chunks)()
    for cname, clevel, shuffle in (("lz4", 1, 1), ("lz4", 5, 2), ("zstd", 1, 1), ("zstd", 3, 2)):
        frames = ctx.compress_device(clevel, shuffle, 2, cname, d.data_ptr(), nb, a.chunks)
        ref = list(pool.map(lambda k: blosc_ref.compress(raw[k * nb:(k + 1) * nb], clevel,
                                                         shuffle, 2, cname), range(a.chunks)))
        assert frames == ref, "frame mismatch"
        ratio = sum(map(len, ref)) / raw.size

        def run_aqz():
            ctx.compress_device(clevel, shuffle, 2, cname, d.data_ptr(), nb, a.chunks,
                                host_dst=dst, dst_stride=stride)

        res = {}
        res["cblosc"] = cpu.cblosc_compress_chunks(raw.ctypes.data, nb, a.chunks, clevel, shuffle,
                                                   2, cname.encode(), a.threads, cdst.ctypes.data,
                                                   nb + 16, csizes, a.reps)
        assert res["cblosc"] > 0, res
        assert [cdst[k * (nb + 16):k * (nb + 16) + csizes[k]].tobytes()
                for k in range(a.chunks)] == ref
        res["cblosc_1thread"] = cpu.cblosc_compress_chunks(
            raw.ctypes.data, nb, a.chunks, clevel, shuffle, 2, cname.encode(), 1,
            cdst.ctypes.data, nb + 16, csizes, 2)
        for name, fn in (("aqz", run_aqz),):
            fn()
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            res[name] = min(ts)
        print(json.dumps({"case": f"{cname} clevel {clevel} shuffle {shuffle}",
                          "chunks": a.chunks, "chunk_bytes": nb, "threads": a.threads,
                          "ratio": round(ratio, 4),
                          "cblosc_ms": round(res["cblosc"] * 1e3, 3),
                          "cblosc_1thread_ms": round(res["cblosc_1thread"] * 1e3, 3),
                          "aqz_ms": round(res["aqz"] * 1e3, 3),
                          "cblosc_GBps": round(raw.size / res["cblosc"] / 1e9, 2),
                          "aqz_GBps": round(raw.size / res["aqz"] / 1e9, 2),
                          "speedup": round(res["cblosc"] / res["aqz"], 2),
                          "codecs": aqz.blosc_codec_info(),
                          "cblosc_version": blosc_ref.version()}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
