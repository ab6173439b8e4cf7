"""Volume Decimate vs Mean over plane shapes with the same bytes per batch
(512 MiB of u16): does the skip pattern of Decimate (every other row, every
other plane) lose HBM channels for some row pitches?  Prints one JSON line
per (shape, method).  A measurement aid, not product code."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import aqz_pkg  # noqa: E402

aqz = aqz_pkg.load()
torch.cuda.set_device(0)
stream = torch.cuda.Stream()
for W, Z in ((512, 1024), (1024, 256), (2048, 64), (4096, 16)):
    H = W
    geo = [(W, H, Z), (W // 2, H // 2, Z // 2), (W // 4, H // 4, Z // 4)]
    d_in = torch.randint(0, 256, (W * H * Z * 2,), dtype=torch.uint8, device="cuda")
    outs = [None] + [torch.empty(w * h * z * 2, dtype=torch.uint8, device="cuda")
                     for w, h, z in geo[1:]]
    ptrs = [0] + [o.data_ptr() for o in outs[1:]]
    torch.cuda.synchronize()
    for mname in ("mean", "decimate"):
        ds = aqz.Downsampler(geo, np.uint16, aqz.METHODS[mname], device=0)
        for _ in range(3):
            counts = ds.run_device_batch(d_in.data_ptr(), Z, ptrs, stream.cuda_stream)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(20):
            ds.run_device_batch(d_in.data_ptr(), Z, ptrs, stream.cuda_stream)
        ev[1].record(stream)
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1e3 / 20
        read = W * H * Z * 2 if mname == "mean" else (Z // 2) * (H // 2) * W * 2
        written = sum(c * w * h * 2 for c, (w, h, _) in zip(counts[1:], geo[1:]))
        print(json.dumps({"W": W, "Z": Z, "method": mname, "kind": ds.last_batch_kind(),
                          "us": round(us, 2), "TBps": round((read + written) / us / 1e6, 3),
                          "frac": round((read + written) / us / 1e6 / 8.0, 4)}), flush=True)
        ds.close()
    del d_in, outs
