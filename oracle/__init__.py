"""ORACLE -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from this package, and only as the checker / the CPU
baseline -- never as the thing measured or shipped.  The product path
(``comapreduce_amd``) never imports it and fails loudly if its HIP library is
missing.

Contents
  oracle.c / liboracle.so   medfilt + binValues restated in C
  l1.py                     Level-1 -> Level-2 reduction restated in NumPy
  destriper.py              destriper (op_Ax, CG, final maps) restated in NumPy
  _ref/libmedfilt_ref.so    the reference's own medianFilter.cpp compiled here

Parity pinning: tests/test_oracle_golden.py checks every restated function
against tests/golden/*.npz, which tests/golden/make_golden.py produced by
running the reference (v0.9.1) itself in the build container.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None


def lib():
    """ctypes handle to oracle/_build/liboracle.so (built on demand with gcc)."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, '_build', 'liboracle.so')
        if not os.path.exists(path):
            subprocess.run(['make', '-C', _HERE, os.path.join(_HERE, '_build', 'liboracle.so')],
                           check=True, stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(path)
        dp = ctypes.POINTER(ctypes.c_double)
        lp = ctypes.POINTER(ctypes.c_int64)
        L.oracle_medfilt.argtypes = [dp, ctypes.c_int64, ctypes.c_int32]
        L.oracle_medfilt.restype = ctypes.c_int
        L.oracle_medfilt_twoheap.argtypes = [dp, ctypes.c_int64, ctypes.c_int32]
        L.oracle_medfilt_twoheap.restype = ctypes.c_int
        L.oracle_bin_values.argtypes = [dp, ctypes.c_int64, lp, dp, lp, ctypes.c_int64]
        L.oracle_bin_values.restype = ctypes.c_int
        _LIB = L
    return _LIB


def ref_lib():
    """The reference's own medianFilter.cpp built by oracle/Makefile (or None)."""
    global _REF
    if _REF is None:
        path = os.path.join(_HERE, '_ref', 'libmedfilt_ref.so')
        if not os.path.exists(path):
            return None
        L = ctypes.CDLL(path)
        fn = getattr(L, '_Z6filterPdii')
        fn.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int]
        fn.restype = None
        _REF = fn
    return _REF


def _dptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def medfilt(x, w):
    """In-place semantics of medfilt.medfilt (medfilt.pyx:26-33); returns the array.

    NaN-free input with n >= w: the order-statistics restatement (oracle_medfilt).
    Input holding NaN, or ceil(w/2) <= n < w: the two-heap restatement
    (oracle_medfilt_twoheap), whose result for NaN follows Mediator.h's insertion
    history as the reference's does."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    if x.size >= w and not np.isnan(x).any():
        rc = lib().oracle_medfilt(_dptr(x), x.size, int(w))
    else:
        rc = lib().oracle_medfilt_twoheap(_dptr(x), x.size, int(w))
    if rc != 0:
        raise ValueError(f'oracle_medfilt failed rc={rc} (n={x.size}, w={w})')
    return x


def medfilt_twoheap(x, w):
    """The two-heap restatement on any input (in place; returns the array)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    rc = lib().oracle_medfilt_twoheap(_dptr(x), x.size, int(w))
    if rc != 0:
        raise ValueError(f'oracle_medfilt_twoheap failed rc={rc} (n={x.size}, w={w})')
    return x


def medfilt_reference(x, w):
    """Runs the reference's compiled filter() (oracle/_ref) in place."""
    fn = ref_lib()
    if fn is None:
        raise RuntimeError('oracle/_ref/libmedfilt_ref.so not built (reference absent)')
    x = np.ascontiguousarray(x, dtype=np.float64)
    fn(_dptr(x), x.size, int(w))
    return x


def bin_values(image, pixels, weights=None, mask=None):
    """binFuncs.binValues (binFuncs.pyx:7-32), in place on ``image``."""
    pixels = np.ascontiguousarray(pixels, dtype=np.int64)
    lp = ctypes.POINTER(ctypes.c_int64)
    w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
    m = None if mask is None else np.ascontiguousarray(mask, dtype=np.int64)
    lib().oracle_bin_values(_dptr(image), image.size, pixels.ctypes.data_as(lp),
                            None if w is None else _dptr(w),
                            None if m is None else m.ctypes.data_as(lp), pixels.size)
    return image
