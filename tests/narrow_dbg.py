"""Debug aid (round 5): the f32 Mean fuzz cases that differ with 16-byte
tiles.  Prints every mismatching output with its 2x2 inputs, under the
test's inputs and with the NaN-payload injection removed.

Round 6: the regression probe of DESIGN.md section 12.1 (run by
tests/test_gpu_divergent.py under round 5's launch environment).
  --cases 4,86     the fuzz cases to run (default: the four round-5 cases)
  --float-mean     every fuzz case of a float type with method Mean
Ends with one line "TOTAL <n> differing outputs"."""
import sys
import os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import torch
import aqz_pkg
import oracle as orc
import test_gpu_fuzz as t
from gpu_util import to_device, empty_device, from_device, launch_stream

aqz = aqz_pkg.load()
torch.cuda.set_device(0)
cases = [4, 86, 174, 192]
if "--cases" in sys.argv:
    cases = [int(c) for c in sys.argv[sys.argv.index("--cases") + 1].split(",")]
if "--float-mean" in sys.argv:
    cases = [i for i in range(t.N_CASES)
             if t.case_params(i)[0] in (np.float32, np.float64) and t.case_params(i)[1] == 1]
total = 0
for case in cases:
    for variant in ("test", "no_payload_nans", "no_specials"):
        dtype, method, w, h, nl, n, in_off, out_off, rng = t.case_params(case)
        geo = t.geometry(w, h, nl)
        if variant != "test" and np.dtype(dtype).kind != "f":
            continue
        if variant == "test":
            frames = t.random_frames(rng, dtype, (n, h, w))
        elif variant == "no_payload_nans":
            frames = t.random_frames(rng, dtype, (n, h, w))
            f = frames.reshape(-1)
            bad = np.isnan(f)
            f[bad] = dtype(np.nan)
        else:
            frames = t.random_frames(rng, dtype, (n, h, w), specials=False)
        exp = t.oracle_stream(orc, geo, dtype, method, frames)
        bpp = np.dtype(dtype).itemsize
        raw = np.zeros(in_off * bpp + frames.nbytes, dtype=np.uint8)
        raw[in_off * bpp:] = frames.view(np.uint8).reshape(-1)
        d_in = to_device(raw)
        outs = [None] + [empty_device((out_off[L] + n * gw * gh) * bpp) for L, (gw, gh, _) in enumerate(geo) if L > 0]
        ptrs = [0] + [outs[L].data_ptr() + out_off[L] * bpp for L in range(1, nl)]
        ds = aqz.Downsampler(geo, dtype, method)
        ds.run_device_batch(d_in.data_ptr() + in_off * bpp, n, ptrs, launch_stream())
        kind = ds.last_batch_kind()
        ds.close()
        nbad = 0
        for L in range(1, nl):
            gw, gh, _ = geo[L]
            got = from_device(outs[L], np.uint8, (-1,))[out_off[L] * bpp:].view(dtype).reshape(n, gh, gw)
            for k, e in enumerate(exp[L]):
                ut = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[bpp]
                gb, eb = got[k].view(ut), e.view(ut)
                diff = np.argwhere(gb != eb)
                nbad += len(diff)
                for (r, c) in diff[:6]:
                    src = frames[k] if L == 1 else None
                    blk = src[2*r:2*r+2, 2*c:2*c+2] if src is not None else None
                    print(f"case {case} {variant} kind {kind} L{L} f{k} r{r} c{c} got {got[k][r,c]!r} want {e[r,c]!r} in {blk.tolist() if blk is not None else ''}")
        total += nbad
        print(f"case {case} {variant}: {nbad} differing outputs ({w}x{h} L{nl} n{n} in_off {in_off} out_off {out_off})", flush=True)
print(f"TOTAL {total} differing outputs", flush=True)
