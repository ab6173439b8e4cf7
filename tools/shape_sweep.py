"""Device-resident pyramid rate over real-world frame shapes (not product).

For each (W, H) it plans the levels like bench.py (chunk 256, 2-D), fills a
batch of >= 1 GiB, times aqz_ds_run_device_batch with HIP events on the
launch stream, and reports GB/s of algorithmic bytes and which batch path
ran (1 fused cascade, 3 batched with single-level kernels, 0 per frame).
The first frame is checked against the oracle.
Usage: python tools/shape_sweep.py [WxH ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402  (binds the HIP runtime first)
import aqz_pkg  # noqa: E402
import oracle  # noqa: E402  (checker only)

SHAPES = ["1920x1080", "2304x2304", "2000x2000", "2048x2048", "4096x4096", "4095x4095",
          "4100x4100", "3000x3000", "2047x2047", "1023x1023", "5120x5120"]


def main(shapes):
    aqz = aqz_pkg.load()
    dtype = np.uint16
    for s in shapes:
        W, H = map(int, s.split("x"))
        dims = [(aqz.TIME, 0, 1, 1), (aqz.SPACE, H, 256, 1), (aqz.SPACE, W, 256, 1)]
        geo = aqz.level_geometry(aqz.plan_levels(dims))
        fb = W * H * 2
        B = max(4, (1 << 30) // fb)
        d_in = torch.randint(0, 256, (B * fb,), dtype=torch.uint8, device="cuda")
        outs = [None] + [torch.empty(B * w * h * 2, dtype=torch.uint8, device="cuda")
                         for w, h, _ in geo[1:]]
        ptrs = [0] + [o.data_ptr() for o in outs[1:]]
        ds = aqz.Downsampler(geo, dtype, aqz.MEAN)
        st = torch.cuda.Stream()
        torch.cuda.synchronize()
        counts = ds.run_device_batch(d_in.data_ptr(), B, ptrs, st.cuda_stream)
        torch.cuda.synchronize()
        # oracle check of frame 0
        f0 = d_in[:fb].cpu().numpy().view(dtype).reshape(H, W)
        ref = oracle.cascade_2d(f0, len(geo), aqz.MEAN)
        ok = all(np.array_equal(outs[L][:geo[L][0] * geo[L][1] * 2].cpu().numpy().view(dtype)
                                .reshape(geo[L][1], geo[L][0]), ref[L - 1])
                 for L in range(1, len(geo)))
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(10)]
        for a, b in ev:
            a.record(st)
            ds.run_device_batch(d_in.data_ptr(), B, ptrs, st.cuda_stream)
            b.record(st)
        torch.cuda.synchronize()
        us = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
        alg = B * fb + sum(counts[L] * geo[L][0] * geo[L][1] * 2 for L in range(1, len(geo)))
        print(f"{s:>10} levels {len(geo)} B {B:4d} kind {ds.last_batch_kind()} "
              f"{us:9.1f} us  {alg / us / 1e3:7.1f} GB/s ({alg / us / 1e3 / 80:.1f}%)  "
              f"{B * W * H / us / 1e3:7.1f} GPix/s  {'bit-exact' if ok else 'MISMATCH'}",
              flush=True)
        ds.close()
        del d_in, outs


if __name__ == "__main__":
    main(sys.argv[1:] or SHAPES)
