"""Drop-in for ``comancpipeline.Tools.median_filter.medfilt`` (medfilt.pyx:26-33).

``medfilt(data, filterSize)`` filters a C-contiguous float64 buffer IN PLACE
and returns it, like the reference's Cython wrapper; the work runs in the
exact chunked sliding-median HIP kernel (comap_medfilt_f64).
"""
import ctypes

import numpy as np

from .. import _native as N


def medfilt(data, filterSize, device=None):
    """``device``: HIP device to run on (default: torch's current device)."""
    if not (isinstance(data, np.ndarray) and data.dtype == np.float64 and data.flags.c_contiguous):
        raise TypeError('medfilt expects a C-contiguous float64 ndarray (double[::1])')
    c = N.ctx(device)
    N.check(N.lib().comap_medfilt_f64(c, N.hptr(data, ctypes.c_double), data.size, int(filterSize)), c,
            'comap_medfilt_f64')
    return data


def medfilt_batch(series, w, reflect=False, device=None):
    """Running median of many series in one device call (comap_medfilt_batch_f64).

    ``reflect=False``: each series exactly as ``medfilt(series, w)``.
    ``reflect=True``: ``medfilt(concat(s[::-1], s, s[::-1]), w)[n:2n]`` -- the
    reflect-padded filters of Level1Averaging.py:696-700 and
    COMAPData.median_filter (COMAPData.py:72-81).  Every series needs n >= w.
    Returns a list of float64 arrays.  ``device``: as for ``medfilt``.
    """
    series = [np.asarray(s, dtype=np.float64) for s in series]
    if not series:
        return []
    offsets = np.zeros(len(series) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum([s.size for s in series])
    x = np.ascontiguousarray(np.concatenate(series))
    out = np.empty_like(x)
    c = N.ctx(device)
    N.check(N.lib().comap_medfilt_batch_f64(c, N.hptr(x, ctypes.c_double), N.hptr(offsets, ctypes.c_int64),
                                            len(series), int(w), 1 if reflect else 0,
                                            N.hptr(out, ctypes.c_double)), c, 'comap_medfilt_batch_f64')
    return [out[offsets[i]:offsets[i + 1]] for i in range(len(series))]
