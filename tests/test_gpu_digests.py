"""Full-size parity against committed digests: every BASELINE config x method
through the HIP path, both the streaming drop-in (add_frame / take_frame)
and the device-resident batch (run_device_batch, the bench path), must hash
to the per-level SHA-256 the REFERENCE ITSELF produced
(tests/golden/reference_digests.json, oracle/_ref).  No CPU code runs here,
so the sizes are the real ones."""
import hashlib
import json

import numpy as np
import pytest

import digest_util as du
from gpu_util import empty_device, launch_stream, to_device, torch_cuda

pytestmark = pytest.mark.gpu

with open(du.GOLDEN) as f:
    GOLD = json.load(f)["configs"]

CASES = [(c, m) for c in du.CONFIGS for m in range(len(du.METHOD_NAMES))]
IDS = [f"{c}-{du.METHOD_NAMES[m]}" for c, m in CASES]


@pytest.mark.parametrize("name,method", CASES, ids=IDS)
def test_stream_matches_digests(aqz, name, method):
    def make(dims, dtype, m):
        geo = aqz.level_geometry(aqz.plan_levels(dims))
        return aqz.Downsampler(geo, dtype, m), geo
    got = du.run_stream(make, name, method)
    assert got == GOLD[name]["methods"][du.METHOD_NAMES[method]]


@pytest.mark.parametrize("name,method", CASES, ids=IDS)
def test_device_batch_matches_digests(aqz, name, method):
    torch = torch_cuda()
    dims, dtype, frames = du.CONFIGS[name]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    W, H, _ = geo[0]
    bpp = np.dtype(dtype).itemsize
    host = np.stack([du.frame(name, k, W, H, dtype) for k in range(frames)])
    d_in = to_device(host)
    outs = [None] + [empty_device(frames * w * h * bpp) for w, h, _ in geo[1:]]
    ds = aqz.Downsampler(geo, dtype, method)
    s = launch_stream()
    counts = ds.run_device_batch(d_in.data_ptr(), frames,
                                 [0] + [o.data_ptr() for o in outs[1:]], s)
    torch.cuda.synchronize()
    kind = ds.last_batch_kind()
    ds.close()
    # the bench configs must take the fused paths (1 cascade, 2 volume)
    assert kind == (2 if len(dims) == 4 else 1), f"batch kind {kind}"
    want = GOLD[name]["methods"][du.METHOD_NAMES[method]]
    for L in range(1, len(geo)):
        w, h, _ = geo[L]
        n = counts[L]
        assert n == want[str(L)]["frames"], f"level {L} frames"
        raw = outs[L][:n * w * h * bpp].cpu().numpy()
        assert hashlib.sha256(raw.tobytes()).hexdigest() == want[str(L)]["sha256"], \
            f"level {L}"
