"""Volume Decimate access-shape A/B (measurement aid, not product code;
VERDICT r4 item 2): tools/volume_probe.hip's variants against the library's
volume_kernel on BASELINE config V (1024 x 1024 x 256 u16, 3 levels),
every output checked against torch slicing, timed with HIP events.

    python tools/volume_probe.py [--reps 30] [--json out.jsonl]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--json", default="")
    ap.add_argument("--W", type=int, default=1024)
    ap.add_argument("--planes", type=int, default=256)
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libaqz_volume_probe.so"))
    vp = ctypes.c_void_p
    u32 = ctypes.c_uint32
    lib.aqz_volume_probe.argtypes = [vp, vp, vp, u32, u32, u32, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, vp]
    import aqz_pkg
    aqz = aqz_pkg.load()
    torch.cuda.set_device(0)
    W = H = a.W
    Z = a.planes
    g = torch.Generator(device="cuda").manual_seed(11)
    src = torch.randint(0, 65536, (Z, H, W), dtype=torch.int32, device="cuda",
                        generator=g).to(torch.int16)
    want1 = src[0::2, 0::2, 0::2].contiguous()
    want2 = src[0::4, 0::4, 0::4].contiguous()
    d1 = torch.empty_like(want1)
    d2 = torch.empty_like(want2)
    stream = torch.cuda.Stream()
    read = (Z // 2) * (H // 2) * W * 2
    written = (d1.numel() + d2.numel()) * 2
    out = open(a.json, "a") if a.json else None

    def timed(launch):
        for _ in range(3):
            launch()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(a.reps):
            launch()
        ev[1].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) * 1e3 / a.reps

    def report(name, us, ok):
        tbps = (read + written) / us / 1e6
        line = {"variant": name, "us": round(us, 2), "TBps": round(tbps, 3),
                "frac": round(tbps / 8.0, 4), "exact": bool(ok)}
        print(json.dumps(line), flush=True)
        if out:
            out.write(json.dumps(line) + "\n")

    # the library's own kernel
    geo = [(W, H, Z), (W // 2, H // 2, Z // 2), (W // 4, H // 4, Z // 4)]
    ds = aqz.Downsampler(geo, np.uint16, aqz.METHODS["decimate"], device=0)
    ptrs = [0, d1.data_ptr(), d2.data_ptr()]
    torch.cuda.synchronize()
    us = timed(lambda: ds.run_device_batch(src.data_ptr(), Z, ptrs, stream.cuda_stream))
    ok = torch.equal(d1, want1) and torch.equal(d2, want2)
    report(f"library kind={ds.last_batch_kind()}", us, ok)
    ds.close()

    for cols in (8, 16):
        for upw in (1, 2, 4, 8):
            for zfast in (0, 1):
                for nt in (1, 0):
                    d1.zero_()
                    d2.zero_()
                    torch.cuda.synchronize()

                    def go():
                        rc = lib.aqz_volume_probe(src.data_ptr(), d1.data_ptr(), d2.data_ptr(),
                                                  W, H, Z, upw, cols, zfast, nt,
                                                  stream.cuda_stream)
                        if rc:
                            raise RuntimeError(f"probe rc {rc}")
                    try:
                        us = timed(go)
                    except RuntimeError:
                        continue
                    ok = torch.equal(d1, want1) and torch.equal(d2, want2)
                    report(f"C{cols} upw{upw} {'zfast' if zfast else 'xfast'} "
                           f"{'nt' if nt else 'plain'}", us, ok)


if __name__ == "__main__":
    main()
