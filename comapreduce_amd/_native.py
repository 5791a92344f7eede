"""ctypes binding of libcomap_hip.so (the C ABI in include/comap_hip.h).

The library is built in-tree by ``__graft_entry__.build()`` /
``make -C comapreduce_amd/csrc`` into ``comapreduce_amd/_lib/``.  There is no
CPU fallback: if the library or a GPU is missing, every op raises.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('COMAP_HIP_LIB') or os.path.join(_HERE, '_lib', 'libcomap_hip.so')

_lib = None
_lock = threading.Lock()
_ctx = {}

c_int, c_int32, c_int64, c_double, c_void_p = ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
P_double = ctypes.POINTER(ctypes.c_double)
P_int32 = ctypes.POINTER(ctypes.c_int32)
P_int64 = ctypes.POINTER(ctypes.c_int64)


class ObsDesc(ctypes.Structure):
    """comap_obs_desc (include/comap_hip.h)."""
    _fields_ = [('n_feeds', c_int32), ('n_bands', c_int32), ('n_channels', c_int32),
                ('n_scans', c_int32), ('n_samples', c_int64), ('tod', c_void_p), ('el', c_void_p),
                ('n_units', c_int32), ('units_host', P_int32)]


# name -> (restype, argtypes)
_SIGS = {
    'comap_ctx_create': (c_int, [c_int, ctypes.POINTER(c_void_p)]),
    'comap_ctx_destroy': (c_int, [c_void_p]),
    'comap_last_error': (ctypes.c_char_p, [c_void_p]),
    'comap_set_stream': (c_int, [c_void_p, c_void_p]),
    'comap_synchronize': (c_int, [c_void_p]),
    'comap_version': (ctypes.c_char_p, []),
    'comap_host_alloc': (c_int, [ctypes.c_size_t, ctypes.POINTER(c_void_p)]),
    'comap_host_free': (None, [c_void_p]),
    'comap_cache_trim': (c_int, []),
    'comap_cache_bytes': (c_int, [P_int64, P_int64, P_int64]),
    'comap_medfilt_f64': (c_int, [c_void_p, P_double, c_int64, c_int32]),
    'comap_medfilt_batch_f64': (c_int, [c_void_p, P_double, P_int64, c_int32, c_int32, c_int32, P_double]),
    'comap_bin_values_f64': (c_int, [c_void_p, P_double, c_int64, P_int64, P_double, P_int64, c_int64]),
    'comap_l1_plan_create': (c_int, [c_void_p, ctypes.POINTER(ObsDesc), ctypes.POINTER(c_void_p)]),
    'comap_l1_plan_destroy': (c_int, [c_void_p]),
    'comap_l1_vane': (c_int, [c_void_p, c_int64, c_int64, P_int32, P_int64, P_int32, P_int64, c_double,
                              c_void_p, c_void_p]),
    'comap_l1_prefetch': (c_int, [c_void_p]),
    'comap_l1_atmosphere': (c_int, [c_void_p, P_int32, c_int32, c_void_p]),
    'comap_l1_average': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    'comap_l1_debug_fetch': (c_int, [c_void_p, c_int32, P_double, c_int64]),
    'comap_l1_channel_bin': (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_l1_profile': (c_int, [c_void_p, c_int32]),
    'comap_l1_profile_collect': (c_int, [c_void_p, P_double, P_int64, c_int32]),
    'comap_spikes': (c_int, [c_void_p, c_void_p, c_int32, c_int64, P_int64, c_int32, c_int32, c_int32, c_double,
                             c_void_p]),
    'comap_power_spectra': (c_int, [c_void_p, c_void_p, c_int32, c_int64, P_int64, c_int32, c_void_p, c_int32,
                                    P_int64, c_void_p]),
    'comap_synth_tod': (c_int, [c_void_p, c_int32, c_int32, c_int64, ctypes.c_uint64, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p]),
    'comap_destripe_create': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int64,
                                      ctypes.POINTER(c_void_p)]),
    'comap_destripe_dist_bin': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_destripe_dist_project': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_destripe_dist_update': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_destripe_dist_direction': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_destripe_dist_parts': (c_int32, []),
    'comap_destripe_dist_project_parts': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                  c_void_p]),
    'comap_destripe_dist_update_fused': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                 c_void_p, c_void_p, c_void_p]),
    'comap_destripe_dist_direction_fused': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_destripe_create_bands': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                            c_int64, c_int32, ctypes.POINTER(c_void_p)]),
    'comap_destripe_create_keyed': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                            c_int64, c_int32, c_int64, c_int32, ctypes.POINTER(c_void_p)]),
    'comap_offset_centroid_keys': (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int64, c_int64, c_void_p, c_int64,
                                           c_void_p]),
    'comap_destripe_destroy': (c_int, [c_void_p]),
    'comap_destripe_n_offsets': (c_int64, [c_void_p]),
    'comap_destripe_n_bands': (c_int32, [c_void_p]),
    'comap_destripe_offsets_natural': (c_int, [c_void_p, c_void_p, c_void_p]),
    'comap_destripe_nnz': (c_int, [c_void_p, P_int64, P_int64]),
    'comap_destripe_entry_bytes': (ctypes.c_int32, [c_void_p]),
    'comap_destripe_sell_entries': (c_int64, [c_void_p]),
    'comap_destripe_local_maps': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_destripe_bin': (c_int, [c_void_p, c_void_p, c_int32, c_void_p]),
    'comap_destripe_project': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_destripe_dot': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_destripe_cg_update': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p]),
    'comap_destripe_cg_direction': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_destripe_div_map': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_relabel_pixels': (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_void_p]),
    'comap_relabel_pixels_tiled': (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int32, c_void_p]),
    'comap_destripe_solve': (c_int, [c_void_p, c_double, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, P_int32]),
    'comap_prep_auto_rms': (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_int64, c_void_p]),
    'comap_prep_percentiles': (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int32, c_int64,
                                       c_void_p]),
    'comap_prep_gather': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    'comap_prep_highpass': (c_int, [c_void_p, c_void_p, c_void_p, c_int32, c_int32]),
    'comap_prep_cut': (c_int, [c_void_p, c_void_p, c_int32, c_int64, c_int32, c_void_p, c_void_p, c_int64,
                               P_int64]),
}

EXPORTED = tuple(_SIGS)


class NativeError(RuntimeError):
    pass


def lib():
    """Load libcomap_hip.so (raises if absent -- there is no fallback)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(f'{LIB_PATH} is missing: build it with '
                                      '`python -c "import __graft_entry__ as g; g.build()"` '
                                      'or `make -C comapreduce_amd/csrc`')
                # torch-ROCm bundles its own libamdhip64.so.7 / libhsa-runtime64: load it first so
                # our NEEDED libamdhip64.so.7 binds to the same (single) HIP runtime in the process;
                # loading /opt/rocm's copy first leaves torch without a device.
                import torch  # noqa: F401
                L = ctypes.CDLL(LIB_PATH)
                for name, (res, args) in _SIGS.items():
                    fn = getattr(L, name)
                    fn.restype = res
                    fn.argtypes = args
                _lib = L
    return _lib


def current_device():
    """torch's current HIP device of this thread (the rank's GPU under torchrun)."""
    import torch
    return torch.cuda.current_device()


def ctx(device=None):
    """Per-process context for ``device`` (default: torch's current device),
    created on first use.  Creating it does not change the current device."""
    if device is None:
        device = current_device()
    device = int(device)
    c = _ctx.get(device)
    if c is None:
        out = c_void_p()
        rc = lib().comap_ctx_create(device, ctypes.byref(out))
        if rc != 0:
            raise NativeError(f'comap_ctx_create(device={device}) failed rc={rc}: no usable HIP device')
        c = out
        _ctx[device] = c
    return c


def check(rc, c=None, what=''):
    if rc != 0:
        msg = lib().comap_last_error(c).decode() if c is not None else ''
        raise NativeError(f'{what} failed rc={rc}: {msg}')
    return rc


def bind_stream(c, torch_device=None):
    """Route the context's work onto torch's current stream (so torch events time it)."""
    import torch
    s = torch.cuda.current_stream(torch_device)
    check(lib().comap_set_stream(c, c_void_p(s.cuda_stream)), c, 'comap_set_stream')


def dptr(t):
    """Device pointer of a contiguous torch CUDA tensor."""
    assert t.is_cuda and t.is_contiguous(), 'expected a contiguous CUDA tensor'
    return c_void_p(t.data_ptr())


def hptr(a, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


class _HostBlock:
    """A cached page-locked block (comap_host_alloc) exposed to NumPy; it returns to
    the cache when the last array viewing it is gone."""

    def __init__(self, shape, dtype):
        import numpy as np
        dt = np.dtype(dtype)
        nbytes = max(int(np.prod(shape)) * dt.itemsize, 1)
        p = c_void_p()
        rc = lib().comap_host_alloc(nbytes, ctypes.byref(p))
        if rc:
            raise MemoryError(f'comap_host_alloc({nbytes}) failed ({rc})')
        self.ptr = p.value
        self.__array_interface__ = {'shape': tuple(int(s) for s in shape), 'typestr': dt.str,
                                    'data': (self.ptr, False), 'version': 3}

    def __del__(self):
        try:
            if self.ptr:
                lib().comap_host_free(c_void_p(self.ptr))
                self.ptr = None
        except Exception:  # pragma: no cover (interpreter shutdown)
            pass


def trim_caches():
    """Return the library's cached device temporaries and page-locked blocks to the
    system (comap_cache_trim) and torch's cached blocks too (torch.cuda.empty_cache)."""
    import torch
    lib().comap_cache_trim()
    torch.cuda.empty_cache()


def cache_bytes():
    """{'device_cached', 'device_live', 'host_cached'} bytes of the library's caches
    (current device)."""
    v = [ctypes.c_int64(0) for _ in range(3)]
    lib().comap_cache_bytes(*(ctypes.byref(x) for x in v))
    return {k: int(x.value) for k, x in zip(('device_cached', 'device_live', 'host_cached'), v)}


def retry_oom(fn, *args, **kw):
    """fn(*args, **kw); on a device out-of-memory (torch's or a native call's) trim the
    caches once and try again."""
    import torch
    try:
        return fn(*args, **kw)
    except (torch.OutOfMemoryError, NativeError) as e:
        if isinstance(e, NativeError) and 'out of memory' not in str(e).lower():
            raise
        trim_caches()
        return fn(*args, **kw)


POISON = os.environ.get('COMAP_POISON') == '1'


def device_empty(shape, dtype, device):
    """Uninitialised device tensor for an output a kernel writes in full: torch.empty,
    retried once after trimming the library's cached temporaries on an out-of-memory
    (the cache may hold memory torch's allocator cannot see).  COMAP_POISON=1 (debug)
    fills it with 0xff bytes -- NaN for floats, -1 for integers -- as the library does
    its own temporaries, so an element no kernel wrote shows up in the results."""
    import torch
    t = retry_oom(torch.empty, shape, dtype=dtype, device=device)
    if POISON:
        if t.is_floating_point():
            t.fill_(float('nan'))
        elif t.dtype == torch.bool:
            t.fill_(True)
        elif t.dtype == torch.uint8:
            t.fill_(255)
        else:
            t.fill_(-1)
    return t


def host_empty(shape, dtype='float64'):
    """Uninitialised page-locked NumPy array from the library's host cache (torch copies
    into it asynchronously: it is pinned memory)."""
    import numpy as np
    return np.asarray(_HostBlock(shape, dtype))

