"""Host-to-host drop-in calls on the headline frame, broken down (measurement
aid, not product code): add_frame alone, add_frame + take_frame of every
level, and add_frame + take_frame_tiled with the tiles made behind the
pyramid (aqz_ds_set_level_tiling) or on demand.  Wall clock per frame.

    python tools/e2e_takes.py [--frames 48] [--shape 4096x4096] [--tile 256]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=48)
    p.add_argument("--shape", default="4096x4096")
    p.add_argument("--tile", type=int, default=256)
    p.add_argument("--levels", type=int, default=5)
    p.add_argument("--only", default="", choices=["", "add", "plain", "behind", "ondemand"])
    p.add_argument("--passes", type=int, default=2)
    a = p.parse_args(argv)
    import aqz_pkg
    aqz = aqz_pkg.load()
    w, h = (int(x) for x in a.shape.split("x"))
    geo = [(w, h, 1)]
    for _ in range(1, a.levels):
        geo.append(((geo[-1][0] + 1) // 2, (geo[-1][1] + 1) // 2, 1))
    rng = np.random.default_rng(0)
    frames = [rng.integers(0, 65536, (h, w), dtype=np.uint16) for _ in range(4)]
    t = a.tile

    def run(label, setup, take):
        ds = aqz.Downsampler(geo, np.uint16, 1)
        setup(ds)
        for i in range(3):
            ds.add_frame(frames[i % 4])
            take(ds)
        t0 = time.perf_counter()
        for i in range(a.frames):
            ds.add_frame(frames[i % 4])
            take(ds)
        ms = (time.perf_counter() - t0) * 1e3 / a.frames
        ds.close()
        print(f"{label}: {ms:.3f} ms/frame", flush=True)

    def no_take(ds):
        pass

    def plain(ds):
        for L in range(1, len(geo)):
            ds.take_frame(L)

    def tiled(ds):
        for L in range(1, len(geo)):
            ds.take_frame_tiled(L, t, t)

    def set_tiling(ds):
        for L in range(1, len(geo)):
            ds.set_level_tiling(L, t, t)

    cases = {"add": ("add_frame only (levels stay cached)", lambda ds: None, no_take),
             "plain": ("add_frame + take_frame", lambda ds: None, plain),
             "behind": ("add_frame + take_frame_tiled, tiled behind the pyramid",
                        set_tiling, tiled),
             "ondemand": ("add_frame + take_frame_tiled, tiled on demand",
                          lambda ds: None, tiled)}
    for _ in range(a.passes):
        for k, c in cases.items():
            if not a.only or a.only == k:
                run(*c)
    return 0


if __name__ == "__main__":
    sys.exit(main())
