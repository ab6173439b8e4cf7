"""Round 6 probe: is the drop-in node mode's per-frame
time against the synchronous drop-in a like-for-like comparison?  The bench's
synchronous leg (`e2e.ms_per_frame`) cycles over 4 pageable frames (128 MiB,
which the host's L3 can hold); its node leg (`e2e.node.dropin_ms_per_frame`)
streams 32 distinct frames (1 GiB).  This times both consumer loops over the
same frame sets, 4 recycled and 32 distinct, on 4096^2 u16, 5 levels, Mean.
Not product code; prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import aqz_pkg  # noqa: E402

aqz = aqz_pkg.load()
W = H = 4096
dims = [(aqz.TIME, 0, 1, 1), (aqz.SPACE, H, 256, 1), (aqz.SPACE, W, 256, 1)]
geo = aqz.level_geometry(aqz.plan_levels(dims))
levels = range(1, len(geo))
rng = np.random.default_rng(5)
distinct = [rng.integers(0, 65535, (H, W), dtype=np.uint16, endpoint=True) for _ in range(32)]
N = 32


def sync_loop(frames):
    ds = aqz.Downsampler(geo, np.uint16, aqz.METHODS["mean"], device=0)
    for i in range(4):
        ds.add_frame(frames[i % len(frames)])
        for L in levels:
            ds.take_frame(L)
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        for i in range(N):
            ds.add_frame(frames[i % len(frames)])
            for L in levels:
                ds.take_frame(L)
        el = (time.perf_counter() - t0) / N
        best = el if best is None else min(best, el)
    ds.close()
    return round(best * 1e3, 3)


def dropin_loop(frames, devices):
    node = aqz.Node(geo, np.uint16, aqz.METHODS["mean"], devices)

    def run():
        for i in range(N):
            node.add_frame(frames[i % len(frames)])
            node.inputs_released()
            for L in levels:
                while node.take_frame(L) is not None:
                    pass
        node.flush()
        for L in levels:
            while node.take_frame(L) is not None:
                pass

    run()
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        run()
        el = (time.perf_counter() - t0) / N
        best = el if best is None else min(best, el)
    node.close()
    return round(best * 1e3, 3)


out = {}
for rep in (1, 2):
    for name, frames in (("recycled4", distinct[:4]), ("distinct32", distinct)):
        out[f"sync_{name}_{rep}"] = sync_loop(frames)
        for devs in ([0], [0, 0]):
            out[f"node{len(devs)}_{name}_{rep}"] = dropin_loop(frames, devs)
print(json.dumps(out))
