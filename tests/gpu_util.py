"""GPU test helpers: device buffers come from torch (plumbing only); every
pyramid computation goes through the native library's C ABI."""
import numpy as np


def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("GPU tests need an AMD GPU (torch.cuda unavailable)")
    return torch


def to_device(arr):
    torch = torch_cuda()
    raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1).copy()
    return torch.from_numpy(raw).to("cuda")


def empty_device(nbytes):
    torch = torch_cuda()
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device="cuda")


def from_device(t, dtype, shape):
    torch_cuda().cuda.synchronize()
    return t.cpu().numpy().view(dtype).reshape(shape)


def random_frames(rng, dtype, shape, specials=True):
    """Full-range integers; floats spread over many magnitudes with NaN, inf,
    -0.0 and denormals injected."""
    dt = np.dtype(dtype)
    if dt.kind in "ui":
        info = np.iinfo(dt)
        return rng.integers(info.min, info.max, size=shape, dtype=dt, endpoint=True)
    x = rng.standard_normal(shape) * np.exp(rng.uniform(-20, 20, shape))
    x = x.astype(dt)
    if specials:
        flat = x.reshape(-1)
        n = flat.size
        k = max(1, n // 200)
        tiny = np.finfo(dt).tiny
        for val in (np.nan, np.inf, -np.inf, -0.0, 0.0, tiny / 8, -tiny / 3):
            idx = rng.integers(0, n, k)
            flat[idx] = dt.type(val)
        # NaNs with random sign and payload, quiet and signaling, written as
        # bits (a float conversion would quiet them): the reference binary's
        # NaN choice must come out byte for byte
        ut = np.dtype(f"u{dt.itemsize}")
        mant = np.finfo(dt).nmant
        bits = flat.view(ut)
        idx = rng.integers(0, n, k)
        exp = ut.type(((1 << (8 * dt.itemsize - 1 - mant)) - 1) << mant)
        sign = rng.integers(0, 2, k).astype(ut) << ut.type(8 * dt.itemsize - 1)
        payload = rng.integers(1, 1 << (mant - 1), k, dtype=np.uint64).astype(ut)
        quiet = (rng.integers(0, 2, k).astype(ut) << ut.type(mant - 1))
        bits[idx] = sign | exp | quiet | payload
    return x


def assert_parity(got, want, ctx=""):
    """Bit-exact for integers; float32/64 within 1 ulp — the tolerance
    north_star states — with NaNs at the same positions carrying the same bits
    (the reference binary's payloads).  The kernels are expected to be
    bit-exact; `exact_fraction` is reported on failure."""
    assert got.shape == want.shape, f"{ctx}: shape {got.shape} vs {want.shape}"
    assert got.dtype == want.dtype
    if got.dtype.kind in "ui":
        if not np.array_equal(got, want):
            bad = np.argwhere(got != want)
            i = tuple(bad[0])
            raise AssertionError(f"{ctx}: {len(bad)} mismatches, first at {i}: "
                                 f"{got[i]} vs {want[i]}")
        return
    gn, wn = np.isnan(got), np.isnan(want)
    assert np.array_equal(gn, wn), f"{ctx}: NaN positions differ"
    ib = np.dtype(f"u{got.dtype.itemsize}")
    assert np.array_equal(got[gn].view(ib), want[wn].view(ib)), f"{ctx}: NaN payloads differ"
    g, w = got[~gn], want[~wn]
    ok = (g == w)
    if not ok.all():
        # within one ulp: got is want or one of its two float neighbours
        up = np.nextafter(w, np.array(np.inf, dtype=w.dtype))
        dn = np.nextafter(w, np.array(-np.inf, dtype=w.dtype))
        near = ok | (g == up) | (g == dn)
        if not near.all():
            i = int(np.argmin(near))
            raise AssertionError(f"{ctx}: {int((~near).sum())} values beyond 1 ulp; "
                                 f"exact fraction {float(ok.mean()):.6f}; first "
                                 f"{g[i]!r} vs {w[i]!r}")


def launch_stream():
    """A non-null torch stream handle for the batch API (NULL would select the
    handle's own stream)."""
    torch = torch_cuda()
    torch.cuda.synchronize()  # inputs were produced on the previous stream
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    return s.cuda_stream
