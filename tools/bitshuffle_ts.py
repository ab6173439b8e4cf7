"""Blosc bit shuffle per typesize against a same-size D2D copy (measurement
aid, not product code).

Streams aqz_blosc_filter_device (BITSHUFFLE, 64 KiB blocks) over successive
32 MiB frames of a resident 1 GiB buffer, as bench.py's secondary_kernels do
for the workload's own dtype, for typesizes 1, 2, 4 and 8, and a D2D copy of
the same bytes; HIP events around each stream of launches.

    python tools/bitshuffle_ts.py [--reps 64]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=64)
    a = p.parse_args(argv)
    import torch
    import aqz_pkg
    aqz = aqz_pkg.load()
    fb = 32 << 20
    nfr = 32
    src = torch.randint(0, 256, (fb * nfr,), dtype=torch.uint8, device="cuda")
    dst = torch.empty(fb, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    sptr = stream.cuda_stream
    base = src.data_ptr()

    def stream_us(launch):
        with torch.cuda.stream(stream):
            for i in range(3):
                launch(i)
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record(stream)
            for i in range(a.reps):
                launch(i)
            e.record(stream)
        torch.cuda.synchronize()
        return b.elapsed_time(e) * 1e3 / a.reps

    copy_us = stream_us(lambda i: dst.copy_(src[(i % nfr) * fb:(i % nfr + 1) * fb]))
    print(f"d2d copy {fb >> 20} MiB: {copy_us:.2f} us/frame "
          f"({2 * fb / copy_us / 1e3:.0f} GB/s)", flush=True)
    for ts in (1, 2, 4, 8):
        us = stream_us(lambda i, ts=ts: aqz.blosc_filter_device(
            aqz.BITSHUFFLE, ts, 65536, base + (i % nfr) * fb, fb, 1, dst.data_ptr(), sptr))
        print(f"bitshuffle ts={ts}: {us:.2f} us/frame ({2 * fb / us / 1e3:.0f} GB/s), "
              f"{copy_us / us:.3f} of the copy", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
