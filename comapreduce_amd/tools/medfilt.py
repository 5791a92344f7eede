"""Drop-in for ``comancpipeline.Tools.median_filter.medfilt`` (medfilt.pyx:26-33).

``medfilt(data, filterSize)`` filters a C-contiguous float64 buffer IN PLACE
and returns it, like the reference's Cython wrapper; the work runs in the
exact chunked sliding-median HIP kernel (comap_medfilt_f64).
"""
import ctypes

import numpy as np

from .. import _native as N


def medfilt(data, filterSize):
    if not (isinstance(data, np.ndarray) and data.dtype == np.float64 and data.flags.c_contiguous):
        raise TypeError('medfilt expects a C-contiguous float64 ndarray (double[::1])')
    c = N.ctx(0)
    N.check(N.lib().comap_medfilt_f64(c, N.hptr(data, ctypes.c_double), data.size, int(filterSize)), c,
            'comap_medfilt_f64')
    return data
