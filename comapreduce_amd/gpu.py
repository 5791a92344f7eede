"""Device-resident observation: the L1 -> L2 hot path on MI355X.

``GPUObservation`` owns the device copy of one Level-1 observation (the f32
cube stays resident in HBM across the three stages) and its
``comap_l1_plan`` (include/comap_hip.h).  The stage classes in
``comapreduce_amd.stages`` are thin wrappers around it; bench.py drives it
directly with device-resident synthetic inputs.

Host work is limited to O(T) control logic the reference also runs on the
host: feature decoding, scan edges, vane sample selection on the 1-D band
average.  Every O(F x 4 x 1024 x T) operation is a HIP kernel; there is no
CPU fallback (missing library or GPU -> exception).
"""
from __future__ import annotations

import ctypes
import time

import numpy as np

from . import _native as N
from .pipeline.datahandling import to_host

N_BANDS, N_CHANNELS = 4, 1024


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise N.NativeError('no HIP device visible to torch: the COMAP hot path has no CPU fallback')
    return torch


def to_device(x, dtype, device):
    """Contiguous CUDA tensor of ``dtype`` (copies host arrays)."""
    torch = _torch()
    if isinstance(x, torch.Tensor):
        t = x.to(device=device, dtype=dtype)
        return t.contiguous()
    if hasattr(x, 'read_flat'):      # a lazy HDF5 dataset (pipeline/h5file.py): staged from the file
        if x.dtype == np.dtype(str(dtype).replace('torch.', '')):
            return upload(x, device)
        x = x[...]
    a = np.ascontiguousarray(to_host(x))
    if a.nbytes >= UPLOAD_MIN_BYTES and a.dtype == np.dtype(str(dtype).replace('torch.', '')):
        return upload(a, device)
    return torch.from_numpy(a).to(device=device, dtype=dtype).contiguous()


UPLOAD_MIN_BYTES = 1 << 28       # host arrays from 256 MB up go through upload()
UPLOAD_CHUNK = 1 << 28           # bytes per pinned staging buffer


def upload(a, device, chunk_bytes=UPLOAD_CHUNK, threads=8):
    """Host array -> device tensor through two pinned staging buffers: host threads
    fill one buffer (np.copyto releases the GIL) while the DMA engine drains the
    other on a copy stream, so a Level-1 cube moves at the PCIe rate instead of a
    pageable copy's.  ``a`` may also be a lazy HDF5 dataset (``read_flat``): the
    native file layer then reads each flat element range straight into the
    staging buffer (the ctypes call releases the GIL, so the copy of the
    previous buffer proceeds meanwhile).  Synchronises before returning."""
    from concurrent.futures import ThreadPoolExecutor
    torch = _torch()
    dev = torch.device(device) if not isinstance(device, int) else torch.device('cuda', device)
    lazy = hasattr(a, 'read_flat')
    if not lazy:
        a = np.ascontiguousarray(a)
    src = None if lazy else a.reshape(-1)
    # the library's cached temporaries are outside torch's allocator: trim them if needed
    out = N.retry_oom(torch.empty, tuple(a.shape), dtype=getattr(torch, str(a.dtype)), device=dev)
    dst = out.view(-1)
    n = int(np.prod(a.shape, dtype=np.int64))
    if n == 0:
        return out
    per = max(1, chunk_bytes // a.dtype.itemsize)
    bufs = [torch.empty(min(per, n), dtype=out.dtype, pin_memory=True) for _ in range(2 if n > per else 1)]
    views = [b.numpy() for b in bufs]
    done = [None] * len(bufs)
    stream = torch.cuda.Stream(dev)
    with ThreadPoolExecutor(threads) as pool:
        for i, off in enumerate(range(0, n, per)):
            k = i % len(bufs)
            m = min(per, n - off)
            if done[k] is not None:
                done[k].synchronize()                      # staging buffer k drained
            if lazy:
                a.read_flat(off, views[k][:m])
            else:
                step = (m + threads - 1) // threads
                list(pool.map(lambda s: np.copyto(views[k][s:min(s + step, m)], src[off + s:off + min(s + step, m)]),
                              range(0, m, step)))
            with torch.cuda.stream(stream):
                dst[off:off + m].copy_(bufs[k][:m], non_blocking=True)
                done[k] = torch.cuda.Event()
                done[k].record(stream)
    stream.synchronize()
    return out


# ---------------------------------------------------------------- vane sample selection (host)
def auto_rms_2d(tod):
    """Tools/stats.py:59-72, 2-D branch (rows = samples)."""
    N2 = (tod.shape[0] // 2) * 2
    return np.nanstd(tod[1:N2:2, :] - tod[:N2:2, :], axis=0) / np.sqrt(2)


def find_hot_cold_from_tod(tod):
    """Hot/cold sample offsets of a vane event from the 1-D band average
    (VaneCalibration.py:86-141); same NumPy operation sequence and dtypes as
    the reference so the selected indices are identical."""
    def find_indices(x, _rms, greater):
        v = x * 1.0
        rng = np.nanmax(v) - np.nanmin(v)
        v /= rng
        rms = _rms / rng
        mid = (np.nanmax(v) + np.nanmin(v)) / 2.0
        cmp = np.greater if greater else np.less
        group = cmp(v - mid, 15 * rms) & (np.abs(np.gradient(v)) < 2e-3)
        return np.arange(v.size, dtype=int)[group]

    rms = auto_rms_2d(tod[:, None]).flatten()
    hot = find_indices(tod, rms, True)
    cold = find_indices(tod, rms, False)
    if len(hot) == 0 or len(cold) == 0:
        return None, None
    hot = np.sort(hot)
    cold = np.sort(cold)
    return hot, cold[cold > hot[-1]]


def find_hot_cold_batch(ba):
    """find_hot_cold_from_tod for every row of ``ba`` [n, L] at once.

    The same NumPy operations as the per-series function, applied along the
    last (contiguous) axis: row reductions use the same pairwise summation and
    the same dtype promotions, so the selected samples are identical (checked
    against the per-series function in tests/test_vane_search.py).  Returns
    (hot, hoff, cold, coff): concatenated int32 sample offsets and int64 row
    offsets; a row where either search comes back empty (the reference's
    RuntimeError path) contributes no samples."""
    x = np.ascontiguousarray(ba)
    n, L = x.shape
    N2 = (L // 2) * 2
    rms0 = np.nanstd(x[:, 1:N2:2] - x[:, :N2:2], axis=1) / np.sqrt(2)
    v = x * 1.0
    rng = np.nanmax(v, axis=1, keepdims=True) - np.nanmin(v, axis=1, keepdims=True)
    v /= rng
    rms = rms0[:, None] / rng
    mid = (np.nanmax(v, axis=1, keepdims=True) + np.nanmin(v, axis=1, keepdims=True)) / 2.0
    flat = np.abs(np.gradient(v, axis=1)) < 2e-3
    hot = np.greater(v - mid, 15 * rms) & flat
    cold = np.less(v - mid, 15 * rms) & flat
    ok = hot.any(axis=1) & cold.any(axis=1)
    col = np.arange(L)
    last_hot = np.where(hot, col, -1).max(axis=1)
    hot &= ok[:, None]
    cold &= ok[:, None] & (col[None, :] > last_hot[:, None])
    hr, hc = np.nonzero(hot)
    cr, cc = np.nonzero(cold)
    hoff = np.zeros(n + 1, dtype=np.int64)
    coff = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(hr, minlength=n), out=hoff[1:])
    np.cumsum(np.bincount(cr, minlength=n), out=coff[1:])
    return hc.astype(np.int32), hoff, cc.astype(np.int32), coff


def vane_events(features):
    """find_vane_samples (VaneCalibration.py:56-65): [[start, end], ...]."""
    flag = features == 13
    idx = np.nonzero(np.diff(flag))[0] + 1
    return idx.reshape((idx.size // 2, 2))


class GPUObservation:
    """One observation resident on one GPU, with its reduction plan."""

    def __init__(self, data, device: int = None):
        torch = _torch()
        device = N.current_device() if device is None else int(device)
        self.device = device
        self.tdev = torch.device('cuda', device)
        self.ctx = N.ctx(device)
        with torch.cuda.device(device):
            self.tod = to_device(data['spectrometer/tod'], torch.float32, self.tdev)
            self.el = to_device(data['spectrometer/pixel_pointing/pixel_el'], torch.float64, self.tdev)
        F, B, C, T = self.tod.shape
        if (B, C) != (N_BANDS, N_CHANNELS):
            raise ValueError(f'unsupported TOD shape {tuple(self.tod.shape)}')
        self.F, self.T = F, T
        self.features = data.features
        self.edges = np.asarray(to_host(data.scan_edges), dtype=np.int64).reshape(-1, 2)
        self.S = len(self.edges)
        self.feeds = np.asarray(to_host(data['spectrometer/feeds'])).reshape(-1)
        units = [(f, s, int(a), int(b - a)) for f in range(F) for s, (a, b) in enumerate(self.edges) if b > a]
        # a shard of a sharded observation (pipeline/sharding.py) reduces only its own units
        filt = getattr(data, 'unit_filter', None)
        if filt is not None:
            keep = {(int(f), int(s)) for f, s in np.asarray(filt).reshape(-1, 2)}
            units = [q for q in units if (q[0], q[1]) in keep]
        if not units:
            raise ValueError('observation (shard) has no (feed, scan) unit to reduce')
        self.units = np.ascontiguousarray(np.array(units, dtype=np.int32).reshape(-1, 4))
        # constant-elevation scans (features == 9 throughout): median atmosphere (Level1Averaging.py:242-244)
        const_scans = {s for s, (a, b) in enumerate(self.edges) if b > a and np.all(self.features[a:b] == 9)}
        self.const_el_units = np.ascontiguousarray(
            np.array([u for u, q in enumerate(self.units) if q[1] in const_scans], dtype=np.int32))
        desc = N.ObsDesc(F, B, C, self.S, T, self.tod.data_ptr(), self.el.data_ptr(), len(units),
                         N.hptr(self.units, ctypes.c_int32))
        plan = ctypes.c_void_p()
        self._bind()
        N.check(N.lib().comap_l1_plan_create(self.ctx, ctypes.byref(desc), ctypes.byref(plan)), self.ctx,
                'comap_l1_plan_create')
        self.plan = plan

    def _bind(self):
        N.bind_stream(self.ctx, self.tdev)

    def close(self):
        if getattr(self, 'plan', None) is not None:
            _torch().cuda.synchronize(self.tdev)
            N.lib().comap_l1_plan_destroy(self.plan)
            self.plan = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass

    # ------------------------------------------------------------ stages
    def vane(self, band_average, t_hot: float, features=None):
        """MeasureSystemTemperature: returns (tsys, gain) CUDA f64 [nV, F, 4, 1024]
        or (None, None) when there is no vane event."""
        torch = _torch()
        feats = self.features if features is None else features
        ev = vane_events(feats)
        nV = ev.shape[0]
        if nV == 0:
            return None, None
        # comap_l1_vane zeroes both before its kernel writes them (no-vane rows stay 0)
        tsys = N.device_empty((nV, self.F, N_BANDS, N_CHANNELS), torch.float64, self.tdev)
        gain = N.device_empty(tuple(tsys.shape), torch.float64, self.tdev)
        self._bind()
        # The band-average windows are copied first (pinned, asynchronous), then pass A
        # (which does not depend on the vane) is queued behind them, so the host search
        # below waits only for the copies and overlaps the 56 GB read.
        windows, copied = [], None
        if isinstance(band_average, torch.Tensor) and band_average.is_cuda:
            for s, e in ev:
                w = torch.empty(tuple(band_average.shape[:2]) + (int(e - s),), dtype=band_average.dtype,
                                pin_memory=True)
                w.copy_(band_average[:, :, s:e], non_blocking=True)
                windows.append(w)
            copied = torch.cuda.Event()
            copied.record()
        else:
            windows = [to_host(band_average[:, :, s:e]) for s, e in ev]
        N.check(N.lib().comap_l1_prefetch(self.plan), self.ctx, 'comap_l1_prefetch')
        t_search = time.perf_counter()
        if copied is not None:
            copied.synchronize()
            windows = [w.numpy() for w in windows]
        for iv, (s, e) in enumerate(ev):
            ba = windows[iv]
            hot, hoff, cold, coff = find_hot_cold_batch(ba.reshape(self.F * N_BANDS, -1))
            self.last_vane_search_ms = (time.perf_counter() - t_search) * 1e3
            N.check(N.lib().comap_l1_vane(self.plan, int(s), int(e - s), N.hptr(hot, ctypes.c_int32),
                                          N.hptr(hoff, ctypes.c_int64), N.hptr(cold, ctypes.c_int32),
                                          N.hptr(coff, ctypes.c_int64), float(t_hot),
                                          N.dptr(tsys[iv]), N.dptr(gain[iv])), self.ctx, 'comap_l1_vane')
        return tsys, gain

    def atmosphere(self):
        """AtmosphereRemoval: CUDA f64 [S, F, 4, 2, 1024]."""
        torch = _torch()
        fit = torch.full((self.S, self.F, N_BANDS, 2, N_CHANNELS), float('nan'), dtype=torch.float64,
                         device=self.tdev)
        self._bind()
        ce = self.const_el_units
        N.check(N.lib().comap_l1_atmosphere(self.plan, N.hptr(ce, ctypes.c_int32) if ce.size else None, int(ce.size),
                                            N.dptr(fit)), self.ctx, 'comap_l1_atmosphere')
        return fit

    def average(self, fit_values, tsys0, gain0, calibrator: bool = False):
        """Level1AveragingGainCorrection: (tod, tod_original, weights) CUDA f64 [F, 4, T]."""
        torch = _torch()
        fit = to_device(fit_values, torch.float64, self.tdev)
        ts = to_device(tsys0, torch.float64, self.tdev)
        gn = to_device(gain0, torch.float64, self.tdev)
        # every sample is written by comap_l1_average (the units' by the reduction, the
        # rest -- scan gaps, a shard's foreign units -- zeroed there)
        out = N.device_empty((3, self.F, N_BANDS, self.T), torch.float64, self.tdev)
        self._bind()
        N.check(N.lib().comap_l1_average(self.plan, N.dptr(fit), N.dptr(ts), N.dptr(gn), int(bool(calibrator)),
                                         N.dptr(out[0]), N.dptr(out[1]), N.dptr(out[2])), self.ctx,
                'comap_l1_average')
        self._keep = (fit, ts, gn)   # inputs must outlive the enqueued kernels
        big = self.feeds > 19        # Level1Averaging.py:817-818
        if big.any():
            out[:, torch.as_tensor(np.flatnonzero(big), device=self.tdev)] = 0
        return out[0], out[1], out[2]

    def channel_bin(self, tsys0, gain0, bin_size: int = 512, mask=None):
        """Level1Averaging.average_tod (Level1Averaging.py:292-321): (avg, stddev) CUDA f64
        [F, 4, 1024 // bin_size, T].  The weights 1/Tsys^2 (zeroed on ``mask``) and their
        per-bin sums are formed on the host with the reference's NumPy expressions (the
        per-bin sum is numpy's pairwise sum over the contiguous bin axis)."""
        torch = _torch()
        if bin_size < 1 or N_CHANNELS % bin_size:
            raise ValueError(f'frequency_bin_size {bin_size} must divide {N_CHANNELS}')
        nb = N_CHANNELS // bin_size
        w = 1.0 / np.asarray(to_host(tsys0), dtype=np.float64).reshape(self.F, N_BANDS, N_CHANNELS) ** 2
        if mask is not None:
            w[..., np.asarray(mask, dtype=bool)] = 0
        wsum = np.sum(w.reshape(self.F, N_BANDS, nb, bin_size), axis=-1)
        wd = to_device(np.ascontiguousarray(w), torch.float64, self.tdev)
        sd = to_device(np.ascontiguousarray(wsum), torch.float64, self.tdev)
        gn = to_device(gain0, torch.float64, self.tdev)
        out = N.device_empty((2, self.F, N_BANDS, nb, self.T), torch.float64, self.tdev)
        self._bind()
        N.check(N.lib().comap_l1_channel_bin(self.plan, int(bin_size), N.dptr(wd), N.dptr(gn), N.dptr(sd),
                                             N.dptr(out[0]), N.dptr(out[1])), self.ctx, 'comap_l1_channel_bin')
        self._keep_bin = (wd, sd, gn)   # inputs must outlive the enqueued kernel
        return out[0], out[1]

    KERNELS = ('vane', 'moments', 'atmos_fit', 'coef_b', 'band_sums', 'median', 'series_sums', 'regress',
               'gain_weights', 'coef_d', 'gain_avg', 'scan_weights', 'unused', 'finish')
    # the HBM streaming passes: A (per-channel moments), B (band means + every per-sample
    # output sum) and C (regression sums); gain_avg is the legacy pass D, launched but idle
    # unless a NaN regression coefficient needs it
    STREAMING = ('moments', 'band_sums', 'regress')

    def profile(self, enable=True):
        """Record HIP events around every kernel launch of this plan (True / 2), around
        the three streaming passes only (1), or not at all (False / 0)."""
        level = 2 if enable is True else int(enable)
        N.check(N.lib().comap_l1_profile(self.plan, level), self.ctx, 'comap_l1_profile')

    def profile_collect(self):
        """{kernel: (total_ms, launches)} since the last collect (synchronises)."""
        ms = np.zeros(32)
        cnt = np.zeros(32, dtype=np.int64)
        N.check(N.lib().comap_l1_profile_collect(self.plan, N.hptr(ms, ctypes.c_double),
                                                 N.hptr(cnt, ctypes.c_int64), 32), self.ctx,
                'comap_l1_profile_collect')
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(self.KERNELS)}

    def pass_fractions(self) -> dict:
        """Fraction of the cube's (unit, band, channel) rows each streaming pass reads:
        A all; B the channel list (median channels with finite alpha); C the list of the
        bands the median filter did not skip.  Rows are weighted by scan length."""
        d = self.debug(9).reshape(-1, 4, 2)
        n = self.units[:, 3].astype(np.float64)[:, None]
        tot = float(n.sum()) * 4 * N_CHANNELS
        return {'moments': 1.0, 'band_sums': float((d[..., 0] * n).sum()) / tot,
                'regress': float((d[..., 0] * d[..., 1] * n).sum()) / tot}

    def scan_samples(self) -> int:
        """Sum over units of the scan lengths (samples each streaming pass visits per channel)."""
        return int(self.units[:, 3].sum())

    def debug(self, what: int):
        """Internal arrays (host f64): 0 rms [U,4,1024]; 1 mf [F,4,T]; 2 dG [F,T]; 3 x [U,4,1024,2]; 4 mb;
        5 kappa [3,U,4,1024]; 6 pass-D sums [U,4,16]; 7 alpha [U,4,1024]; 8 atmosphere (o, a) [U,4,1024,2];
        9 per (unit, band): channel-list length, median band on [U,4,2]."""
        U = self.units.shape[0]
        shapes = {0: (U, 4, 1024), 1: (self.F, 4, self.T), 2: (self.F, self.T), 3: (U, 4, 1024, 2),
                  4: (self.F, 4, self.T), 5: (3, U, 4, 1024), 6: (U, 4, 16), 7: (U, 4, 1024), 8: (U, 4, 1024, 2),
                  9: (U, 4, 2)}
        out = np.empty(shapes[what])
        self._bind()
        N.check(N.lib().comap_l1_debug_fetch(self.plan, what, N.hptr(out, ctypes.c_double), out.size), self.ctx,
                'comap_l1_debug_fetch')
        return out


def gpu_observation(data, device: int = None) -> GPUObservation:
    """The GPUObservation cached on a Level-1 data object (created on first use);
    ``device`` None = torch's current device."""
    device = N.current_device() if device is None else int(device)
    obs = getattr(data, '_gpu_observation', None)
    if obs is None or obs.device != device:
        obs = GPUObservation(data, device)
        data._gpu_observation = obs
    return obs
