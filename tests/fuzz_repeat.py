"""Round 6 probe: run device-batch fuzz cases many times
in one process and count the runs with a wrong output, per case.  Used on
the edge-load probe builds (tools/divergent/, $AQZ_LIB_PATH); the checker is
the oracle, so this lives with the tests.
  python tests/fuzz_repeat.py --cases 181 --reps 100 [--from 0]
--from K first runs cases K..(first case - 1) once, as the fuzz suite would
before it.  Prints one JSON line: {case: [bad runs, runs, [first values]]}."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import torch  # noqa: E402
import aqz_pkg  # noqa: E402
import oracle as orc  # noqa: E402
import test_gpu_fuzz as t  # noqa: E402
from gpu_util import to_device, empty_device, from_device, launch_stream  # noqa: E402

aqz = aqz_pkg.load()
torch.cuda.set_device(0)
args = sys.argv[1:]
cases = [int(c) for c in args[args.index("--cases") + 1].split(",")] if "--cases" in args else [181]
reps = int(args[args.index("--reps") + 1]) if "--reps" in args else 50
start = int(args[args.index("--from") + 1]) if "--from" in args else None


def prepare(case):
    dtype, method, w, h, nl, n, in_off, out_off, rng = t.case_params(case)
    geo = t.geometry(w, h, nl)
    frames = t.random_frames(rng, dtype, (n, h, w))
    exp = t.oracle_stream(orc, geo, dtype, method, frames)
    return dtype, method, geo, nl, n, in_off, out_off, frames, exp


def run(prep):
    dtype, method, geo, nl, n, in_off, out_off, frames, exp = prep
    bpp = np.dtype(dtype).itemsize
    raw = np.zeros(in_off * bpp + frames.nbytes, dtype=np.uint8)
    raw[in_off * bpp:] = frames.view(np.uint8).reshape(-1)
    d_in = to_device(raw)
    outs = [None] + [empty_device((out_off[L] + n * gw * gh) * bpp)
                     for L, (gw, gh, _) in enumerate(geo) if L > 0]
    ptrs = [0] + [outs[L].data_ptr() + out_off[L] * bpp for L in range(1, nl)]
    ds = aqz.Downsampler(geo, dtype, method)
    ds.run_device_batch(d_in.data_ptr() + in_off * bpp, n, ptrs, launch_stream())
    ds.close()
    bad = []
    ut = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[bpp]
    for L in range(1, nl):
        gw, gh, _ = geo[L]
        got = from_device(outs[L], np.uint8, (-1,))[out_off[L] * bpp:].view(dtype).reshape(n, gh, gw)
        for k, e in enumerate(exp[L]):
            d = np.argwhere(got[k].view(ut) != e.view(ut))
            for r, c in d[:2]:
                bad.append([L, k, int(r), int(c), got[k][r, c].item(), e[r, c].item()])
    return bad


if start is not None:
    for c in range(start, min(cases)):
        run(prepare(c))
out = {}
preps = {c: prepare(c) for c in cases}
for c in cases:
    nbad, first = 0, []
    for _ in range(reps):
        b = run(preps[c])
        if b:
            nbad += 1
            if len(first) < 3:
                first.append(b[0])
    out[c] = [nbad, reps, first]
print(json.dumps(out))
