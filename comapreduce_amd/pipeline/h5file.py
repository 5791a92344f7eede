"""HDF5 files through the native file layer (include/comap_h5.h, libcomap_h5.so).

The reference does all of its file I/O with h5py (DataHandling.py:101-179,
COMAPData.py:170-435); h5py is not in this image, libhdf5 is.  ``H5File`` is
the small h5py-shaped surface the pipeline needs: ``visit`` (visititems'
objects), ``read`` / ``dataset`` (a lazy ``H5Dataset`` for the large
``spectrometer/tod``, sliced by hyperslab), ``write`` (intermediate groups
created, an existing object replaced), attributes with h5py's value types
(numeric scalars as NumPy scalars, str for variable-length strings, bytes for
fixed-length ones, arrays otherwise).  No torch import: this is host I/O.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get('COMAP_H5_LIB') or os.path.join(_HERE, '_lib', 'libcomap_h5.so')
MAX_RANK = 32

# include/comap_h5.h enum comap_h5_dtype
F32, F64, I8, I16, I32, I64, U8, U16, U32, U64, BOOL, STR_FIXED, STR_VLEN = range(1, 14)
_CODE_OF = {np.dtype(np.float32): F32, np.dtype(np.float64): F64, np.dtype(np.int8): I8, np.dtype(np.int16): I16,
            np.dtype(np.int32): I32, np.dtype(np.int64): I64, np.dtype(np.uint8): U8, np.dtype(np.uint16): U16,
            np.dtype(np.uint32): U32, np.dtype(np.uint64): U64, np.dtype(np.bool_): BOOL}
_DTYPE_OF = {v: k for k, v in _CODE_OF.items()}

_lib = None
_lock = threading.Lock()

c_int, c_int32, c_int64, c_void_p, c_char_p = ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_char_p
P_i32, P_i64 = ctypes.POINTER(c_int32), ctypes.POINTER(c_int64)
_SIGS = {
    'comap_h5_version': (c_char_p, []),
    'comap_h5_last_error': (c_char_p, []),
    'comap_h5_open': (c_int, [c_char_p, c_int32, ctypes.POINTER(c_void_p)]),
    'comap_h5_close': (c_int, [c_void_p]),
    'comap_h5_flush': (c_int, [c_void_p]),
    'comap_h5_exists': (c_int, [c_void_p, c_char_p]),
    'comap_h5_visit': (c_int64, [c_void_p, c_char_p, c_int64]),
    'comap_h5_require_group': (c_int, [c_void_p, c_char_p]),
    'comap_h5_delete': (c_int, [c_void_p, c_char_p]),
    'comap_h5_info': (c_int, [c_void_p, c_char_p, P_i32, P_i32, P_i64, P_i64]),
    'comap_h5_read': (c_int, [c_void_p, c_char_p, c_int32, c_int64, P_i64, P_i64, c_void_p]),
    'comap_h5_read_flat': (c_int, [c_void_p, c_char_p, c_int32, c_int64, c_int64, c_int64, c_void_p]),
    'comap_h5_write': (c_int, [c_void_p, c_char_p, c_int32, c_int64, c_int32, P_i64, c_void_p]),
    'comap_h5_read_strings': (c_int64, [c_void_p, c_char_p, c_char_p, c_char_p, c_int64]),
    'comap_h5_write_strings': (c_int, [c_void_p, c_char_p, c_char_p, c_int32, P_i64, c_char_p]),
    'comap_h5_attr_list': (c_int64, [c_void_p, c_char_p, c_char_p, c_int64]),
    'comap_h5_attr_info': (c_int, [c_void_p, c_char_p, c_char_p, P_i32, P_i32, P_i64, P_i64]),
    'comap_h5_attr_read': (c_int, [c_void_p, c_char_p, c_char_p, c_int32, c_int64, c_void_p]),
    'comap_h5_attr_write': (c_int, [c_void_p, c_char_p, c_char_p, c_int32, c_int64, c_int32, P_i64, c_void_p]),
}
EXPORTED = tuple(_SIGS)


class H5Error(RuntimeError):
    pass


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib():
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise H5Error(f'{LIB_PATH} is missing: build it with __graft_entry__.build() '
                              '(needs libhdf5 headers under /opt/conda)')
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                fn = getattr(L, name)
                fn.restype, fn.argtypes = res, args
            _lib = L
    return _lib


def _check(rc, what):
    if rc < 0:
        raise H5Error(f'{what}: {lib().comap_h5_last_error().decode(errors="replace")}')
    return rc


def _b(s):
    return s.encode() if isinstance(s, str) else s


def _text(call, *args):
    """Calls a (..., buf, cap) -> needed listing function (needed counts the
    terminating NUL) with a big enough buffer."""
    n = _check(call(*args, None, 0), 'listing')
    buf = ctypes.create_string_buffer(int(n) + 1)
    _check(call(*args, buf, len(buf)), 'listing')
    return buf.raw[:max(0, n - 1)]


def _shape(nd, dims):
    return tuple(int(dims[i]) for i in range(nd.value))


def _np_dtype(code, elsize):
    if code == STR_FIXED:
        return np.dtype(f'S{int(elsize)}')
    if code in _DTYPE_OF:
        return _DTYPE_OF[code]
    raise H5Error(f'unsupported HDF5 type code {code}')


def _to_writable(value):
    """(kind, array) for a value to store: kind 'vlen' (str data) or 'plain'."""
    if isinstance(value, str):
        return 'vlen', np.array(value, dtype=object)
    if isinstance(value, bytes):
        return 'plain', np.array(value, dtype=f'S{max(1, len(value))}')
    a = np.asarray(value)
    if a.dtype.kind == 'U' or (a.dtype == object and a.size and all(isinstance(x, str) for x in a.reshape(-1))):
        return 'vlen', a.astype(object)
    if a.dtype == object and a.size == 0:
        return 'vlen', a
    if a.dtype.kind == 'S':
        return 'plain', a if a.dtype.itemsize > 0 else a.astype('S1')
    if a.dtype.kind == 'c':
        raise H5Error('complex datasets are not supported')
    if a.dtype.byteorder == '>':
        a = a.astype(a.dtype.newbyteorder('='))
    if a.dtype not in _CODE_OF:
        raise H5Error(f'unsupported dtype {a.dtype}')
    return 'plain', a


def _pack_strings(a):
    return b''.join(str(x).encode('utf-8') + b'\0' for x in a.reshape(-1))


def _unpack_strings(raw, shape):
    parts = raw.split(b'\0')[:-1] if raw else []
    vals = [p.decode('utf-8', errors='surrogateescape') for p in parts]
    if not shape:
        return vals[0] if vals else ''
    out = np.empty(len(vals), dtype=object)
    out[:] = vals
    return out.reshape(shape)


class H5File:
    """An open HDF5 file (mode 'r', 'a' or 'w', as h5py.File)."""

    def __init__(self, filename: str, mode: str = 'r'):
        modes = {'r': 0, 'a': 1, 'r+': 1, 'w': 2}
        if mode not in modes:
            raise ValueError(f'mode {mode!r}')
        if mode == 'r+' and not os.path.exists(filename):
            raise FileNotFoundError(filename)
        h = c_void_p()
        _check(lib().comap_h5_open(_b(filename), modes[mode], ctypes.byref(h)), f'open {filename}')
        self._h = h
        self.filename = filename
        self.mode = mode

    # ------------------------------------------------------------ lifetime
    def close(self):
        h, self._h = getattr(self, '_h', None), None
        if h:
            _check(lib().comap_h5_close(h), f'close {self.filename}')

    def reopen(self):
        """Re-open a closed read-only file on the same object, so every lazy
        dataset / row view taken from it (here or in a shard) works again after
        the file was closed for a rewrite (HDF5Data.write_data_file)."""
        if self._h:
            return
        if self.mode != 'r':
            raise H5Error(f'{self.filename}: only read-only files are re-opened')
        h = c_void_p()
        _check(lib().comap_h5_open(_b(self.filename), 0, ctypes.byref(h)), f'open {self.filename}')
        self._h = h

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass

    @property
    def handle(self):
        if not self._h:
            raise H5Error(f'{self.filename} is closed')
        return self._h

    # ------------------------------------------------------------ structure
    def __contains__(self, path):
        return _check(lib().comap_h5_exists(self.handle, _b(path)), 'exists') == 1

    def visit(self):
        """[(path, 'dataset'|'group')] of every object below the root (visititems)."""
        out = []
        for line in _text(lib().comap_h5_visit, self.handle).decode().splitlines():
            kind, path = line.split(' ', 1)
            out.append((path, 'dataset' if kind == 'D' else 'group'))
        return out

    def require_group(self, path):
        _check(lib().comap_h5_require_group(self.handle, _b(path)), f'group {path}')

    def delete(self, path):
        _check(lib().comap_h5_delete(self.handle, _b(path)), f'delete {path}')

    # ------------------------------------------------------------ datasets
    def info(self, path):
        """(dtype code, shape, element size)."""
        code, nd, es = c_int32(), c_int32(), c_int64()
        dims = (c_int64 * MAX_RANK)()
        _check(lib().comap_h5_info(self.handle, _b(path), ctypes.byref(code), ctypes.byref(nd), dims,
                                   ctypes.byref(es)), f'info {path}')
        return code.value, _shape(nd, dims), es.value

    def dataset(self, path) -> 'H5Dataset':
        return H5Dataset(self, path)

    def read(self, path):
        """The whole dataset as a NumPy array (0-d for scalars; object array of str
        for variable-length strings)."""
        code, shape, es = self.info(path)
        if code == STR_VLEN:
            return _unpack_strings(_text_strings(self, path, None), shape)
        out = np.empty(shape, dtype=_np_dtype(code, es))
        _check(lib().comap_h5_read(self.handle, _b(path), code, es, None, None, out.ctypes.data_as(c_void_p)),
               f'read {path}')
        return out

    def write(self, path, value):
        kind, a = _to_writable(value)
        dims = (c_int64 * max(1, a.ndim))(*a.shape)
        if kind == 'vlen':
            _check(lib().comap_h5_write_strings(self.handle, _b(path), None, a.ndim, dims, _pack_strings(a)),
                   f'write {path}')
            return
        a = np.require(a, requirements="C")   # (ascontiguousarray would make 0-d arrays 1-d)
        code = STR_FIXED if a.dtype.kind == 'S' else _CODE_OF[a.dtype]
        _check(lib().comap_h5_write(self.handle, _b(path), code, a.dtype.itemsize, a.ndim, dims,
                                    a.ctypes.data_as(c_void_p)), f'write {path}')

    # ------------------------------------------------------------ attributes
    def attr_names(self, path):
        return _text(lib().comap_h5_attr_list, self.handle, _b(path)).decode().splitlines()

    def attrs(self, path) -> dict:
        return {k: self.attr(path, k) for k in self.attr_names(path)}

    def attr(self, path, name):
        code, nd, es = c_int32(), c_int32(), c_int64()
        dims = (c_int64 * MAX_RANK)()
        _check(lib().comap_h5_attr_info(self.handle, _b(path), _b(name), ctypes.byref(code), ctypes.byref(nd), dims,
                                        ctypes.byref(es)), f'attribute {path}:{name}')
        shape = _shape(nd, dims)
        if code.value == STR_VLEN:
            return _unpack_strings(_text_strings(self, path, name), shape)
        out = np.empty(shape, dtype=_np_dtype(code.value, es.value))
        _check(lib().comap_h5_attr_read(self.handle, _b(path), _b(name), code.value, es.value,
                                        out.ctypes.data_as(c_void_p)), f'attribute {path}:{name}')
        return out[()] if out.ndim == 0 else out

    def set_attr(self, path, name, value):
        kind, a = _to_writable(value)
        dims = (c_int64 * max(1, a.ndim))(*a.shape)
        if kind == 'vlen':
            _check(lib().comap_h5_write_strings(self.handle, _b(path), _b(name), a.ndim, dims, _pack_strings(a)),
                   f'attribute {path}:{name}')
            return
        a = np.require(a, requirements="C")   # (ascontiguousarray would make 0-d arrays 1-d)
        code = STR_FIXED if a.dtype.kind == 'S' else _CODE_OF[a.dtype]
        _check(lib().comap_h5_attr_write(self.handle, _b(path), _b(name), code, a.dtype.itemsize, a.ndim, dims,
                                         a.ctypes.data_as(c_void_p)), f'attribute {path}:{name}')


def _text_strings(f, path, attr):
    L = lib()
    n = _check(L.comap_h5_read_strings(f.handle, _b(path), _b(attr) if attr else None, None, 0), 'strings')
    buf = ctypes.create_string_buffer(max(1, int(n)))
    _check(L.comap_h5_read_strings(f.handle, _b(path), _b(attr) if attr else None, buf, len(buf)), 'strings')
    return buf.raw[:n]


class H5Dataset:
    """Lazy dataset (what h5py hands the reference for ``large_datasets``):
    shape/dtype without reading, basic slicing by hyperslab, and flat element
    ranges (``read_flat``) for the staged host->device upload."""

    def __init__(self, f: H5File, path: str):
        self.file, self.name = f, path
        self._code, self.shape, self._es = f.info(path)
        if self._code == STR_VLEN:
            raise H5Error(f'{path}: lazy variable-length string datasets are not supported')
        self.dtype = _np_dtype(self._code, self._es)

    ndim = property(lambda s: len(s.shape))
    size = property(lambda s: int(np.prod(s.shape, dtype=np.int64)))
    nbytes = property(lambda s: s.size * s.dtype.itemsize)

    def __len__(self):
        if not self.shape:
            raise TypeError('len() of a scalar dataset')
        return self.shape[0]

    def __array__(self, dtype=None, copy=None):
        a = self[...]
        return a if dtype is None else a.astype(dtype)

    def read_flat(self, offset: int, out: np.ndarray) -> np.ndarray:
        """out[:] = flattened dataset[offset : offset + out.size] (out contiguous, this dtype)."""
        if out.dtype != self.dtype or not out.flags.c_contiguous:
            raise ValueError('read_flat needs a contiguous buffer of the dataset dtype')
        _check(lib().comap_h5_read_flat(self.file.handle, _b(self.name), self._code, self._es, int(offset),
                                        int(out.size), out.ctypes.data_as(c_void_p)), f'read {self.name}')
        return out

    def __getitem__(self, key):
        if not isinstance(key, tuple):
            key = (key,)
        if any(k is Ellipsis for k in key):
            i = next(j for j, k in enumerate(key) if k is Ellipsis)
            fill = (slice(None),) * (self.ndim - (len(key) - 1))
            key = key[:i] + fill + key[i + 1:]
        if len(key) > self.ndim:
            raise IndexError('too many indices')
        key = key + (slice(None),) * (self.ndim - len(key))
        start, count, post, squeeze = [], [], [], []
        for ax, (k, n) in enumerate(zip(key, self.shape)):
            if isinstance(k, (int, np.integer)):
                i = int(k) + (n if k < 0 else 0)
                if not 0 <= i < n:
                    raise IndexError(f'index {k} out of range for axis {ax} of size {n}')
                start.append(i); count.append(1); post.append(slice(None)); squeeze.append(ax)
            elif isinstance(k, slice):
                lo, hi, st = k.indices(n)
                if st < 0:                      # read the covering range, reverse afterwards
                    lo2, hi2 = (hi + 1, lo + 1) if hi < lo else (0, 0)
                    start.append(lo2); count.append(max(0, hi2 - lo2))
                    post.append(slice(None, None, st) if count[-1] else slice(0, 0))
                else:
                    hi = max(hi, lo)
                    start.append(lo); count.append(hi - lo); post.append(slice(None, None, st))
            elif ax == 0 and np.ndim(k) == 1 and np.asarray(k).dtype.kind in 'iu':
                # integer list on the leading axis (e.g. a feed selection): one hyperslab
                # read per listed row, never the whole dataset
                rows = [self[(int(i),) + tuple(key[1:])] for i in np.asarray(k)]
                return np.stack(rows) if rows else np.empty((0,) + self[(0,) + tuple(key[1:])].shape, self.dtype)
            else:
                a = np.asarray(self)[tuple(key)]   # other fancy indexing: read, then index
                return a
        out = np.empty(tuple(count), dtype=self.dtype)
        if out.size:
            s = (c_int64 * max(1, self.ndim))(*start)
            c = (c_int64 * max(1, self.ndim))(*count)
            _check(lib().comap_h5_read(self.file.handle, _b(self.name), self._code, self._es, s, c,
                                       out.ctypes.data_as(c_void_p)), f'read {self.name}')
        out = out[tuple(post)]
        if squeeze:
            out = out.reshape([m for ax, m in enumerate(out.shape) if ax not in squeeze])
        return out

    def rows(self, lo: int, hi: int) -> 'H5Rows':
        """Lazy view of rows [lo, hi) of the leading axis (a feed range of a cube)."""
        return H5Rows(self, lo, hi)

    def __repr__(self):
        return f'<H5Dataset {self.name!r}: shape {self.shape}, dtype {self.dtype}>'


class H5Rows:
    """Rows [lo, hi) of a lazy dataset's leading axis, still lazy: what a shard
    of a file-backed observation holds (pipeline/sharding.slice_feeds), so only
    its own feeds are read from the file when it is staged to the device."""

    def __init__(self, ds: H5Dataset, lo: int, hi: int):
        n = ds.shape[0]
        lo, hi, _ = slice(lo, hi).indices(n)
        self.ds, self.lo, self.hi = ds, lo, max(lo, hi)
        self.shape = (self.hi - self.lo,) + tuple(ds.shape[1:])
        self.dtype = ds.dtype
        self._inner = int(np.prod(ds.shape[1:], dtype=np.int64))

    ndim = property(lambda s: len(s.shape))
    size = property(lambda s: int(np.prod(s.shape, dtype=np.int64)))
    nbytes = property(lambda s: s.size * s.dtype.itemsize)

    def __len__(self):
        return self.shape[0]

    def read_flat(self, offset: int, out: np.ndarray) -> np.ndarray:
        if offset < 0 or offset + out.size > self.size:
            raise IndexError('flat range out of the view')
        return self.ds.read_flat(self.lo * self._inner + int(offset), out)

    def rows(self, lo: int, hi: int) -> 'H5Rows':
        lo, hi, _ = slice(lo, hi).indices(self.shape[0])
        return H5Rows(self.ds, self.lo + lo, self.lo + max(lo, hi))

    def __array__(self, dtype=None, copy=None):
        a = self.ds[self.lo:self.hi]
        return a if dtype is None else a.astype(dtype)

    def __getitem__(self, key):
        return np.asarray(self)[key]
