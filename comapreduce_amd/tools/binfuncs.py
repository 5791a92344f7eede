"""Drop-in for ``comancpipeline.Tools.binFuncs.binValues`` (binFuncs.pyx:7-32).

``binValues(image, pixels, weights=None, mask=None)`` accumulates in place:
image[p] += weights[i] (or += 1) for 0 <= p < image.size and mask[i] != 0.
The device path sorts samples by pixel (stable) and adds each pixel's
contributions in sample order, so results are bit-identical to the
reference's serial loop.
"""
import ctypes

import numpy as np

from .. import _native as N


def binValues(image, pixels, weights=None, mask=None, device=None):
    """``device``: HIP device to run on (default: torch's current device)."""
    if not (isinstance(image, np.ndarray) and image.dtype == np.float64 and image.flags.c_contiguous):
        raise TypeError('image must be a C-contiguous float64 ndarray')
    pix = np.ascontiguousarray(pixels, dtype=np.int64)
    w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
    m = None if mask is None else np.ascontiguousarray(mask, dtype=np.int64)
    if w is not None and w.size != pix.size:
        raise ValueError('weights and pixels differ in length')
    c = N.ctx(device)
    N.check(N.lib().comap_bin_values_f64(c, N.hptr(image, ctypes.c_double), image.size,
                                         N.hptr(pix, ctypes.c_int64),
                                         None if w is None else N.hptr(w, ctypes.c_double),
                                         None if m is None else N.hptr(m, ctypes.c_int64), pix.size),
            c, 'comap_bin_values_f64')
