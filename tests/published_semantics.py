"""numpy restatements of the third-party reductions the reference's Python
tests compare against (python/tests/test_stream.py:993-1190).

The reference names them in its OME metadata (downsampler.cpp:440-485):
  skimage.transform.downscale_local_mean(x, (2, 2), cval=0)   scikit-image 0.25.2
  skimage.measure.block_reduce(x, (2, 2), func=np.min|np.max) scikit-image 0.25.2
  x[::2, ::2]                                                  numpy 2.2.6
scikit-image is not installed here, so their published algorithms are
restated: a block reduction over 2x2 blocks after padding the right/bottom
edge with `cval` (0) to a multiple of the block, computed in float64 for the
mean.  The Python tests use them only on even-sized frames, where no padding
happens; that is the only regime used below.
"""
import numpy as np


def _blocks(x):
    h, w = x.shape
    assert h % 2 == 0 and w % 2 == 0, "restatement covers even frames only"
    return x.reshape(h // 2, 2, w // 2, 2)


def downscale_local_mean(x):
    return _blocks(x.astype(np.float64)).mean(axis=(1, 3))


def block_reduce_min(x):
    return _blocks(x).min(axis=(1, 3))


def block_reduce_max(x):
    return _blocks(x).max(axis=(1, 3))


def decimate(x):
    return x[::2, ::2]
