"""GPU parity against vectors made by the REFERENCE ITSELF
(tests/golden/reference_vectors.{npz,json}: acquire-zarr v0.8.1's
zarr::Downsampler compiled unmodified, tests/golden/make_reference_vectors.py).

* the streaming drop-in (aqz_ds_add_frame / aqz_ds_take_frame) replays all
  400 cases — 10 geometries x 10 dtypes x 4 methods — frame by frame, with the
  reference's frame readiness, untaken frames and odd-Z pass-through; two of
  the geometries are BASELINE config C1a itself (the reference example's 5-D
  t10 c8 z6 y48 x64 array and its frames i*1000+j: the 10 frames the example
  appends, and one whole timepoint);
* the device batch (aqz_ds_run_device_batch, the bench path) reproduces each
  level's frames of every geometry whose levels are all taken after every
  frame.

Every case is compared byte for byte, floats included: NaN payloads must be
the ones the reference binary made (x86's first-NaN-operand rule and its
negative default NaN, restated in ds_kernels.hip's x86_add).  The
NaN-payload set (reference_nan_vectors.npz: inputs dense in quiet and
signaling NaNs of both signs and random payloads, and infinities) replays the
same way.  No reference code runs here — the fixtures travel, the reference
does not.
"""
import numpy as np
import pytest

import refvec as rv
from gpu_util import empty_device, from_device, launch_stream, to_device, torch_cuda

pytestmark = pytest.mark.gpu

MAN, VEC = rv.load()
NAN_VEC = np.load(rv.NAN_NPZ, allow_pickle=False)
CASES = rv.cases(MAN)
IDS = [f"{g}-{d}-{rv.METHOD_NAMES[m]}" for g, d, m in CASES]
NAN_CASES = rv.nan_cases()
NAN_IDS = [f"nan-{g}-{d}-{rv.METHOD_NAMES[m]}" for g, d, m in NAN_CASES]


def _stream_replay(aqz, vec, geom, dtype, method):
    handles = []

    def make(dims, dt, m):
        ds = aqz.Downsampler(aqz.level_geometry(aqz.plan_levels(dims)), dt, m)
        handles.append(ds)
        return ds
    try:
        rv.replay(make, MAN, vec, geom, dtype, method, nan_bits=True)
    finally:
        for ds in handles:
            ds.close()


@pytest.mark.parametrize("geom,dtype,method", CASES, ids=IDS)
def test_stream_replays_reference_vectors(aqz, geom, dtype, method):
    _stream_replay(aqz, VEC, geom, dtype, method)


@pytest.mark.parametrize("geom,dtype,method", NAN_CASES, ids=NAN_IDS)
def test_stream_replays_reference_nan_vectors(aqz, geom, dtype, method):
    _stream_replay(aqz, NAN_VEC, geom, dtype, method)


BATCH_CASES = [("main", g, d, m) for g, d, m in CASES
               if MAN["geometries"][g]["take"] == "all"]
BATCH_CASES += [("nan", g, d, m) for g, d, m in NAN_CASES
                if MAN["geometries"][g]["take"] == "all"]


@pytest.mark.parametrize("vset,geom,dtype,method", BATCH_CASES,
                         ids=[f"{v}-{g}-{d}-{rv.METHOD_NAMES[m]}" for v, g, d, m in BATCH_CASES])
def test_device_batch_reproduces_reference_levels(aqz, vset, geom, dtype, method):
    torch = torch_cuda()
    vec = VEC if vset == "main" else NAN_VEC
    g = MAN["geometries"][geom]
    dt = np.dtype(dtype)
    frames = vec[f"in/{geom}/{dtype}"]
    name = f"{geom}/{dtype}/{rv.METHOD_NAMES[method]}"
    ev, out = vec[f"ev/{name}"], vec[f"out/{name}"]
    # the reference's frames per level, in emit order
    want = {L: [] for L in range(1, len(g["levels"]))}
    off = 0
    for k, L, has, nb in ev:
        if has:
            want[int(L)].append(out[off:off + nb])
            off += int(nb)
    geo = [tuple(x) for x in g["geometry"]]
    n = frames.shape[0]
    bpp = dt.itemsize
    d_in = to_device(frames)
    outs = [None] + [empty_device(n * w * h * bpp) for w, h, _ in geo[1:]]
    ds = aqz.Downsampler(geo, dt, method)
    try:
        counts = ds.run_device_batch(d_in.data_ptr(), n, [0] + [o.data_ptr() for o in outs[1:]],
                                     launch_stream())
        torch.cuda.synchronize()
    finally:
        ds.close()
    for L, frames_L in want.items():
        w, h, _ = geo[L]
        assert counts[L] == len(frames_L), f"{name}: level {L} frames"
        got = from_device(outs[L], np.uint8, (-1,))[:len(frames_L) * w * h * bpp]
        for k, wb in enumerate(frames_L):
            gb = got[k * w * h * bpp:(k + 1) * w * h * bpp]
            bad = rv.same(gb, wb, dt, nan_bits=True)
            assert bad is None, f"{name}: level {L} frame {k}: {bad.size} elements differ"
