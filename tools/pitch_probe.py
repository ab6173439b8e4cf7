"""What the frame pitch alone costs HBM (measurement aid, not product code).

Runs tools/hbm_probe.hip's row-shaped probe (aqz_hbm_probe_rows: the
cascade's 16-row x 1 KiB wave units, loads only, 16:5 contiguous nt stores)
over about 2 GiB of dense u16 frames of each shape, with and without
nontemporal loads, timed with HIP events on one stream.  The aligned
headline rows (8192 B) against rows that split 128-B lines (3000^2: 6000 B,
5472x3648: 10944 B, 2000^2: 4000 B) give the pitch penalty a kernel with this
read pattern cannot avoid; bench.py --shape gives the kernel's own rate on
the same box.

    python tools/pitch_probe.py [--reps 20] [--json out.jsonl] [--set volume]

--set volume runs the volume kernel's read patterns instead: every row of
every plane (Mean), and every other row of every other plane (Decimate), for
square u16 planes 512-4096 wide.  --set decimate: 2-D Decimate's every-other-
row reads against all rows, for 512^2 u8, 2048^2 and 4096^2 u16 frames.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SHAPES = [(4096, 4096), (3000, 3000), (5472, 3648), (2000, 2000),
          (2048, 2048), (1920, 1080)]


def frame_cases():
    """Dense u16 frames: (label, row_bytes, pitch, rows, frame_stride)."""
    return [(f"{w}x{h}", w * 2, w * 2, h, w * 2 * h) for w, h in SHAPES]


def volume_cases():
    """The volume kernel's reads for square u16 planes of width w: Mean reads
    every row of every plane; Decimate every other row (pitch 2 rows) of
    every other plane (frame stride 2 planes)."""
    out = []
    for w in (512, 1024, 2048, 4096):
        rb, plane = w * 2, w * 2 * w
        out.append((f"plane{w}_all_rows", rb, rb, w, plane))
        out.append((f"plane{w}_decimate", rb, 2 * rb, w // 2, 2 * plane))
    return out


def decimate_cases():
    """Decimate's 2-D read pattern (every other row) against all rows, for
    the 512^2 u8 frames of config C1b (512-B rows: the skipped half of every
    1 KiB pair of rows is the neighbour of what is read) and the 4096^2 u16
    headline (8 KiB rows), VERDICT r3 item 5."""
    out = []
    for label, rb, h in (("512x512_u8", 512, 512), ("4096x4096_u16", 8192, 4096),
                         ("2048x2048_u16", 4096, 2048)):
        out.append((f"{label}_all_rows", rb, rb, h, rb * h))
        out.append((f"{label}_decimate", rb, 2 * rb, h // 2, rb * h))
    return out


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--gib", type=float, default=2.0)
    p.add_argument("--json", default="")
    p.add_argument("--set", default="frames", choices=["frames", "volume", "decimate"],
                   help="frames: dense u16 frames of SHAPES; volume: the volume "
                        "kernel's Mean and Decimate read patterns")
    a = p.parse_args(argv)
    import torch
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libaqz_hbm_probe.so"))
    f = lib.aqz_hbm_probe_rows
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                  ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    total = int(a.gib * (1 << 30))
    src = torch.randint(0, 256, (total + (1 << 20),), dtype=torch.uint8, device="cuda")
    sink = torch.zeros(16, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    out = open(a.json, "w") if a.json else None
    cases = {"volume": volume_cases, "decimate": decimate_cases}.get(a.set, frame_cases)()
    for label, row_bytes, pitch, h, fstride in cases:
        frames = max(1, total // fstride)
        units = frames * (-(-h // 16)) * (-(-row_bytes // 1024))
        dst = torch.empty(units * 5 * 1024, dtype=torch.uint8, device="cuda")
        res = {"shape": label, "row_bytes": row_bytes, "pitch": pitch, "frames": frames,
               "row_bytes_mod_128": row_bytes % 128}
        for nt in (1, 0):
            for wr in (5, 0):
                moved = ctypes.c_uint64(0)

                def go():
                    rc = f(src.data_ptr(), row_bytes, pitch, h, fstride, frames,
                           dst.data_ptr(), sink.data_ptr(), wr, nt,
                           ctypes.c_void_p(stream.cuda_stream), ctypes.byref(moved))
                    if rc:
                        raise RuntimeError(f"aqz_hbm_probe_rows: {rc}")
                with torch.cuda.stream(stream):
                    for _ in range(3):
                        go()
                    ev = [(torch.cuda.Event(enable_timing=True),
                           torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
                    for b, e in ev:
                        b.record(stream)
                        go()
                        e.record(stream)
                torch.cuda.synchronize()
                us = sum(b.elapsed_time(e) for b, e in ev) / len(ev) * 1e3
                key = ("nt" if nt else "cached") + ("_rw16to5" if wr else "_read")
                res[key + "_us"] = round(us, 2)
                res[key + "_GBps"] = round(moved.value / (us * 1e-6) / 1e9, 1)
        del dst
        line = json.dumps(res)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
    if out:
        out.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
