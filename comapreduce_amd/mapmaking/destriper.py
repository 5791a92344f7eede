"""Destriping map-maker on MI355X (drop-in for comancpipeline/MapMaking/Destriper.py).

``run_destriper`` keeps the reference signature and return value
(Destriper.py:456-503): ``{'All': {'map', 'naive', 'weight', 'map2', 'hits'}}``
on rank 0 and ``None`` maps on other ranks.  Internally:

* ``DeviceOps`` -- one rank's samples as the constant offset<->pixel sparse
  operator built by ``comap_destripe_create`` (destriper_kernels.hip);
* ``cg_solve`` -- the reference BiCG (Destriper.py:85-152) with its two
  duplicate matvecs folded (p == pb, r == rb), run on device vectors; per
  iteration the only exchange is a SUM all-reduce of the map numerator
  (npix f64) and of two scalars (p.q, r.r) -- RCCL over xGMI when
  torch.distributed is initialised with the nccl backend.  ``cg_solve`` is
  backend-agnostic (the gloo CPU tests drive it with the oracle's NumPy ops).

Samples are sharded by whole offsets (the reference shards files,
run_destriper.py:131-138); the map is replicated.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .. import _native as N


def _dist():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist
    except ImportError:  # pragma: no cover
        pass
    return None


def torch_allreduce(t):
    """SUM all-reduce in place (no-op on one rank)."""
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(t, op=d.ReduceOp.SUM)
    return t


class TimedAllreduce:
    """torch_allreduce with every call bracketed by HIP events on the current stream (the
    stream the CG kernels run on, which waits for the collective): the measured
    all-reduce time and bytes per CG iteration that mapmaking/rankplan.py's alpha / beta
    are calibrated from (bench.py, N > 1).  The first ``skip`` calls (the set-up sums of
    h, the naive numerator and rr0 in cg_solve_batched) are recorded apart."""

    def __init__(self, skip=3):
        self.calls, self.skip = [], skip

    def __call__(self, t):
        import torch
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch_allreduce(t)
        e1.record()
        self.calls.append((t.numel() * t.element_size(), e0, e1))
        return t

    def summary(self, iterations):
        import torch
        torch.cuda.synchronize()
        body = self.calls[self.skip:]
        ms = [a.elapsed_time(b) for _, a, b in body]
        it = max(int(iterations), 1)
        per = len(body) // it if body else 0
        sizes = [n for n, _, _ in body[:per]]
        by_call = [sum(ms[k::per]) / it for k in range(per)] if per else []
        return {'iterations': it, 'calls_per_iter': per, 'bytes_per_call': sizes,
                'ms_per_call': by_call, 'allreduce_ms_per_iter': sum(ms) / it,
                'bytes_per_iter': sum(sizes)}


def compact_pixels(pix, npix, allreduce):
    """(pixel ids relabelled onto the union over ranks of the pixels the operator touches,
    int32; the union's pixel ids, increasing).  The union holds every binned pixel and
    every pixel an unbinned sample reads: op_Z reads m[pointing] (Destriper.py:206-213),
    so a negative id p reads pixel npix + p.  Such a sample keeps a negative id in the
    compacted map of nc pixels, cid[npix + p] - nc, which reads the same pixel there.
    pix: int64 torch tensor on any device (ids in [-npix, npix)); allreduce sums in place."""
    import torch
    read = torch.remainder(pix, npix)            # the pixel each sample bins or reads
    hit = torch.zeros(npix, dtype=torch.int32, device=pix.device)
    hit[read] = 1
    allreduce(hit)
    keep = hit > 0
    cid = torch.cumsum(keep.to(torch.int64), 0) - 1
    nc = int(keep.sum().item())
    comp = torch.where(pix >= 0, cid[read], cid[read] - nc)
    return comp.to(torch.int32), torch.nonzero(keep).reshape(-1)


def cg_solve(ops, allreduce, threshold=1e-6, niter=100, h=None, nnum=None):
    """Distributed CG for the destriper offsets.

    ops: operator object (DeviceOps or oracle.destriper.ShardOps) for this
    rank's samples; allreduce(array) sums in place across ranks.  h / nnum
    are the global weight map and naive numerator (computed when None).
    Returns (x, iterations, h, nnum); for DeviceOps x is in the problem's internal
    offset order (DeviceOps.natural converts)."""
    if getattr(ops, 'nb', 1) != 1:
        raise ValueError('cg_solve drives one band; batched bands use cg_solve_batched')
    if h is None or nnum is None:
        h0, _, n0 = ops.local_maps()
        h = allreduce(h0)
        nnum = allreduce(n0)
    NO = ops.n_offsets
    x = ops.zeros(NO)
    r = ops.zeros(NO)
    ops.project(None, nnum, h, r)                # b = op_Ax(tod, extend=False); r0 = b - A 0
    p = ops.copy(r)
    rr0 = ops.scalar()
    ops.dot(r, r, rr0)
    allreduce(rr0)
    rr = ops.copy(rr0)
    thresh0 = ops.host_scalar(rr0)
    num = ops.zeros(ops.npix)
    q = ops.zeros(NO)
    pq = ops.scalar()
    rrn = ops.scalar()
    it = 0
    for i in range(niter):
        ops.bin(p, 0, num)
        allreduce(num)
        ops.project(p, num, h, q, pq)
        allreduce(pq)
        ops.cg_update(rr, pq, x, r, p, q, rrn)
        allreduce(rrn)
        ops.cg_direction(rrn, rr, p, r)
        ops.set_scalar(rr, rrn)
        it = i + 1
        delta = ops.host_scalar(rrn) / thresh0
        if np.isnan(delta) or delta < threshold:
            break
    return x, it, h, nnum


def cg_solve_batched(ops, allreduce, threshold=1e-6, niter=100, batch=16):
    """Multi-rank CG of the device path: the iterates of ``cg_solve`` (same
    order of operations and cross-rank sums), but with the convergence test on
    the device (comap_destripe_dist_direction's stop flags) so ``batch``
    iterations -- kernels and all-reduces -- are queued per host round trip.
    Iterations queued after convergence are no-ops (their all-reduces sum
    stale buffers that are not read again).  Works for every band of a batched
    problem at once (vectors interleaved [n][nb], one all-reduce per sum for
    all bands).  Returns (x in the problem's internal offset order -- see
    DeviceOps.natural --, iterations per band (list), h, nnum)."""
    torch = ops.torch
    nb = ops.nb
    h0, _, n0 = ops.local_maps()
    h = allreduce(h0)
    nnum = allreduce(n0)
    NO = ops.n_offsets
    x, r, q = ops.zeros(NO * nb), ops.zeros(NO * nb), ops.zeros(NO * nb)
    num = ops.zeros(ops.npix * nb)
    ops.project(None, nnum, h, r)
    p = ops.copy(r)
    scal = ops.zeros(4 * nb + 1)        # rr0, rr, pq, rr_new (nb each), threshold
    ops.dot(r, r, scal[0:nb])
    allreduce(scal[0:nb])
    scal[nb:2 * nb].copy_(scal[0:nb])
    scal[3 * nb:4 * nb].copy_(scal[0:nb])
    scal[4 * nb] = float(threshold)
    flags = torch.zeros(2 + 2 * nb, dtype=torch.int32, device=ops.dev)
    iteration = _dist_iteration(ops, allreduce, p, num, h, q, scal, flags, x, r)
    enq = 0
    while enq < niter:
        k = min(batch, niter - enq)
        for _ in range(k):
            iteration()
        enq += k
        if int(flags[0].item()):
            break
    return x, [int(v) for v in flags[2 + nb:2 + 2 * nb].tolist()], h, nnum


def _dist_iteration(ops, allreduce, p, num, h, q, scal, flags, x, r):
    """One multi-rank CG iteration as a no-argument callable: by default the native
    solve's 4 kernels with the p.q / r.r block partials all-reduced
    (comap_destripe_dist_*_parts / _fused); COMAP_DS_DIST_FUSED=0 (and operator
    objects without them, e.g. the oracle's) use the 7-launch pieces that all-reduce
    final sums."""
    nb = ops.nb
    if hasattr(ops, 'dist_parts') and os.environ.get('COMAP_DS_DIST_FUSED', '1') != '0':
        pq_part, rr_part = ops.dist_parts()

        def fused():
            ops.dist_bin(p, num, flags)
            allreduce(num)
            ops.dist_project_parts(p, num, h, q, pq_part, flags)
            allreduce(pq_part)
            ops.dist_update_fused(scal, pq_part, x, r, p, q, rr_part, flags)
            allreduce(rr_part)
            ops.dist_direction_fused(scal, rr_part, p, r, flags)
        return fused

    def pieces():
        ops.dist_bin(p, num, flags)
        allreduce(num)
        ops.dist_project(p, num, h, q, scal, flags)
        allreduce(scal[2 * nb:3 * nb])
        ops.dist_update(scal, x, r, p, q, flags)
        allreduce(scal[3 * nb:4 * nb])
        ops.dist_direction(scal, p, r, flags)
    return pieces


def cg_solve_graph(ops, allreduce, threshold=1e-6, niter=100, batch=16):
    """cg_solve_batched with each batch of ``batch`` iterations -- the four kernel
    pieces AND the three all-reduces of every iteration -- captured once into a
    HIP graph (torch.cuda.graph; RCCL collectives are capturable) and replayed:
    one graph launch per batch instead of 7 host calls per iteration.  Same
    iterates, bit for bit, as cg_solve_batched (same kernels, same sums).  The
    remainder niter % batch runs eagerly.  Returns like cg_solve_batched."""
    torch = ops.torch
    nb = ops.nb
    h0, _, n0 = ops.local_maps()
    h = allreduce(h0)
    nnum = allreduce(n0)
    NO = ops.n_offsets
    x, r, q = ops.zeros(NO * nb), ops.zeros(NO * nb), ops.zeros(NO * nb)
    num = ops.zeros(ops.npix * nb)
    ops.project(None, nnum, h, r)
    p = ops.copy(r)
    scal = ops.zeros(4 * nb + 1)
    ops.dot(r, r, scal[0:nb])
    allreduce(scal[0:nb])
    scal[nb:2 * nb].copy_(scal[0:nb])
    scal[3 * nb:4 * nb].copy_(scal[0:nb])
    scal[4 * nb] = float(threshold)
    flags = torch.zeros(2 + 2 * nb, dtype=torch.int32, device=ops.dev)
    iteration = _dist_iteration(ops, allreduce, p, num, h, q, scal, flags, x, r)

    nfull = niter // batch
    graph = None
    if nfull:
        side = torch.cuda.Stream(ops.dev)
        side.wait_stream(torch.cuda.current_stream(ops.dev))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=side):
            for _ in range(batch):
                iteration()
    done = 0
    for _ in range(nfull):
        graph.replay()
        done += batch
        if int(flags[0].item()):
            break
    if not int(flags[0].item()):
        for _ in range(niter - done):
            iteration()
    return x, [int(v) for v in flags[2 + nb:2 + 2 * nb].tolist()], h, nnum


class DeviceOps:
    """One rank's destriper operator on the GPU (comap_destripe_* C ABI).

    ``tod``/``weights`` are [N] (one band) or [n_bands, N] (several sidebands on
    the same ``pixels``, solved as one batched system -- comap_destripe_create_bands;
    3 bands are padded to 4 with an empty band).  ``keep`` (optional, [n_bands,
    N/L]) marks the offsets each band's data prep kept.  Per-band vectors are
    interleaved band-fastest ([N/L][nb], [npix][nb])."""

    def __init__(self, pixels, tod, weights, offset_length, npix, device=None, keep=None, okey=None):
        """okey (optional): (int32 CUDA [N/L] keys, exclusive bound) -- the offsets' internal
        processing order (comap_destripe_create_keyed); default: each offset's first on-map
        pixel."""
        import torch
        self.torch = torch
        device = N.current_device() if device is None else int(device)
        self.dev = torch.device('cuda', device)
        self.ctx = N.ctx(device)
        self.pix = self._t(pixels, torch.int32)
        tod2 = self._t2(tod, torch.float64)
        w2 = self._t2(weights, torch.float64)
        self.n_bands = int(tod2.shape[0])           # bands the caller asked for
        if w2.shape != tod2.shape:
            raise ValueError('tod and weights must have the same shape')
        if self.n_bands not in (1, 2, 3, 4):
            raise ValueError('1 to 4 bands per problem')
        self.nb = 4 if self.n_bands == 3 else self.n_bands
        n = int(tod2.shape[1])
        if self.pix.numel() != n:
            raise ValueError('pointing, tod and weights must have the same length')
        if n % offset_length:
            raise ValueError('number of samples must be a multiple of offset_length')
        # (pixel indices >= npix are caught by the set-up's count pass on the device: rc -3)
        self.L, self.npix = int(offset_length), int(npix)
        kp = None
        if keep is not None:
            kp = self._t2(keep, torch.uint8)
            if kp.shape != (self.n_bands, n // self.L):
                raise ValueError('keep must be [n_bands, n_samples // offset_length]')
        if self.nb != self.n_bands:              # pad 3 -> 4 bands with an empty band
            z = torch.zeros((1, n), dtype=torch.float64, device=self.dev)
            tod2, w2 = torch.cat([tod2, z]), torch.cat([w2, z])
            if kp is not None:
                kp = torch.cat([kp, torch.zeros((1, n // self.L), dtype=torch.uint8, device=self.dev)])
        self.tod, self.w, self.keep = tod2.contiguous(), w2.contiguous(), kp
        h = ctypes.c_void_p()
        N.bind_stream(self.ctx, self.dev)
        keys, kmax = okey if okey is not None else (None, 0)
        if keys is not None and (keys.numel() != n // self.L or keys.dtype != torch.int32):
            raise ValueError('okey must be int32 [n_samples // offset_length]')
        rc = N.lib().comap_destripe_create_keyed(self.ctx, N.dptr(self.pix), N.dptr(self.tod), N.dptr(self.w),
                                                 None if kp is None else N.dptr(kp),
                                                 None if keys is None else N.dptr(keys), int(kmax), n, self.L,
                                                 self.npix, self.nb, ctypes.byref(h))
        if rc == -3:
            raise IndexError(f'pixel index out of range for a map of {npix} pixels (valid: -{npix} .. {npix - 1})')
        N.check(rc, self.ctx, 'comap_destripe_create_bands')
        self.h = h
        self.n_offsets = int(N.lib().comap_destripe_n_offsets(h))

    def _t(self, a, dt):
        torch = self.torch
        if isinstance(a, torch.Tensor):
            return a.to(device=self.dev, dtype=dt).contiguous().reshape(-1)
        return torch.from_numpy(np.ascontiguousarray(a)).to(device=self.dev, dtype=dt).reshape(-1)

    def _t2(self, a, dt):
        torch = self.torch
        t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
        t = t.to(device=self.dev, dtype=dt)
        return t.reshape(1, -1).contiguous() if t.dim() == 1 else t.contiguous()

    def natural(self, x):
        """Offset vector in the caller's offset order (the C side processes offsets in
        a spatially sorted internal order; every other vector here is internal)."""
        out = self.zeros(self.n_offsets * self.nb)
        self._c('comap_destripe_offsets_natural', self.h, self._v(x), self._v(out))
        return out

    def split_bands(self, v):
        """[n*nb] interleaved -> [n_bands, n] (contiguous copy, padding band dropped)."""
        return v.reshape(-1, self.nb).t()[:self.n_bands].contiguous()

    def __del__(self):
        try:
            if getattr(self, 'h', None) is not None:
                self.torch.cuda.synchronize(self.dev)
                N.lib().comap_destripe_destroy(self.h)
                self.h = None
        except Exception:  # pragma: no cover
            pass

    def nnz(self):
        a = ctypes.c_int64()
        b = ctypes.c_int64()
        N.lib().comap_destripe_nnz(self.h, ctypes.byref(a), ctypes.byref(b))
        return int(a.value), int(b.value)

    def entry_bytes(self):
        """Bytes per operator entry: 4 + NB (count form) or 4 + 8 NB."""
        return int(N.lib().comap_destripe_entry_bytes(self.h))

    def sell_entries(self):
        """Padded entries of the projection's sliced-ELLPACK rows (-1: none)."""
        return int(N.lib().comap_destripe_sell_entries(self.h))

    # ---- vector helpers
    def empty(self, n):
        """[n] float64 on the device, uninitialised (for outputs a call writes in full)."""
        return N.device_empty(n, self.torch.float64, self.dev)

    def zeros(self, n):
        return self.torch.zeros(n, dtype=self.torch.float64, device=self.dev)

    def scalar(self):
        return self.zeros(1)

    def copy(self, a):
        return a.clone()

    def host_scalar(self, s):
        return float(s.item())

    def set_scalar(self, dst, src):
        dst.copy_(src)

    def _c(self, fn, *args):
        N.bind_stream(self.ctx, self.dev)
        N.check(getattr(N.lib(), fn)(*args), self.ctx, fn)

    # ---- operand checks: every device buffer handed to the C ABI must hold what the
    # kernels index (offset vectors [N/L * nb], maps [npix * nb], nb scalars, ...)
    def _v(self, t):
        if t.numel() < self.n_offsets * self.nb or t.dtype != self.torch.float64:
            raise ValueError(f'offset vector must be float64 with >= {self.n_offsets * self.nb} values')
        return N.dptr(t)

    def _m(self, t):
        if t.numel() < self.npix * self.nb or t.dtype != self.torch.float64:
            raise ValueError(f'map must be float64 with >= {self.npix * self.nb} values')
        return N.dptr(t)

    def _s(self, t, n=None):
        n = self.nb if n is None else n
        if t.numel() < n or t.dtype != self.torch.float64:
            raise ValueError(f'scalar buffer must be float64 with >= {n} values')
        return N.dptr(t)

    def _f(self, t):
        if t.numel() < 2 + 2 * self.nb or t.dtype != self.torch.int32:
            raise ValueError(f'flags must be int32 with >= {2 + 2 * self.nb} values')
        return N.dptr(t)

    # ---- operator pieces
    def local_maps(self):
        h, hits, nn = (self.zeros(self.npix * self.nb) for _ in range(3))
        self._c('comap_destripe_local_maps', self.h, self._m(h), self._m(hits), self._m(nn))
        return h, hits, nn

    def bin(self, x, mode, out):
        self._c('comap_destripe_bin', self.h, self._v(x), int(mode), self._m(out))

    def project(self, x, num, h, y, dot=None):
        self._c('comap_destripe_project', self.h, None if x is None else self._v(x), self._m(num), self._m(h),
                self._v(y), None if dot is None else self._s(dot))

    def dot(self, a, b, out):
        self._c('comap_destripe_dot', self.h, self._v(a), self._v(b), self._s(out))

    def cg_update(self, rr, pq, x, r, p, q, rr_new):
        self._c('comap_destripe_cg_update', self.h, self._s(rr), self._s(pq), self._v(x), self._v(r), self._v(p),
                self._v(q), self._s(rr_new))

    def cg_direction(self, rr_new, rr, p, r):
        self._c('comap_destripe_cg_direction', self.h, self._s(rr_new), self._s(rr), self._v(p), self._v(r))

    # ---- multi-rank iteration pieces (device stop flags; see cg_solve_batched)
    def dist_bin(self, p, num, flags):
        self._c('comap_destripe_dist_bin', self.h, self._v(p), self._m(num), self._f(flags))

    def dist_project(self, p, num, h, q, scal, flags):
        self._c('comap_destripe_dist_project', self.h, self._v(p), self._m(num), self._m(h), self._v(q),
                self._s(scal, 4 * self.nb + 1), self._f(flags))

    def dist_update(self, scal, x, r, p, q, flags):
        self._c('comap_destripe_dist_update', self.h, self._s(scal, 4 * self.nb + 1), self._v(x), self._v(r),
                self._v(p), self._v(q), self._f(flags))

    def dist_direction(self, scal, p, r, flags):
        self._c('comap_destripe_dist_direction', self.h, self._s(scal, 4 * self.nb + 1), self._v(p), self._v(r),
                self._f(flags))

    # ---- the same iteration with block partials all-reduced (4 launches, as the native solve)
    def dist_parts(self):
        """Zeroed [nb * comap_destripe_dist_parts()] partial buffers for p.q and r.r."""
        n = int(N.lib().comap_destripe_dist_parts()) * self.nb
        return self.zeros(n), self.zeros(n)

    def _pp(self, t):
        n = int(N.lib().comap_destripe_dist_parts()) * self.nb
        if t.numel() < n or t.dtype != self.torch.float64:
            raise ValueError(f'partial buffer must be float64 with >= {n} values')
        return N.dptr(t)

    def dist_project_parts(self, p, num, h, q, pq_part, flags):
        self._c('comap_destripe_dist_project_parts', self.h, self._v(p), self._m(num), self._m(h), self._v(q),
                self._pp(pq_part), self._f(flags))

    def dist_update_fused(self, scal, pq_part, x, r, p, q, rr_part, flags):
        self._c('comap_destripe_dist_update_fused', self.h, self._s(scal, 4 * self.nb + 1), self._pp(pq_part),
                self._v(x), self._v(r), self._v(p), self._v(q), self._pp(rr_part), self._f(flags))

    def dist_direction_fused(self, scal, rr_part, p, r, flags):
        self._c('comap_destripe_dist_direction_fused', self.h, self._s(scal, 4 * self.nb + 1), self._pp(rr_part),
                self._v(p), self._v(r), self._f(flags))

    def div_map(self, num, h, out):
        self._c('comap_destripe_div_map', self.h, self._m(num), self._m(h), self._m(out))

    # ---- single-rank native solve (no Python per iteration)
    def solve_native(self, threshold, niter):
        """x [N/L * nb], iterations per band (list), maps {k: [npix * nb]} (interleaved)."""
        nb = self.nb
        x = self.empty(self.n_offsets * nb)                  # the solve writes x and every map in full
        maps = {k: self.empty(self.npix * nb) for k in ('map', 'naive', 'weight', 'hits')}
        it = (ctypes.c_int32 * nb)()
        self._c('comap_destripe_solve', self.h, float(threshold), int(niter), N.dptr(x), N.dptr(maps['map']),
                N.dptr(maps['naive']), N.dptr(maps['weight']), N.dptr(maps['hits']),
                ctypes.cast(it, ctypes.POINTER(ctypes.c_int32)))
        return x, [int(v) for v in it][:self.n_bands], maps

    def solve_native_host(self, threshold, niter, unmap=None):
        """solve_native with the maps delivered to the host: {k: NumPy [n_bands, npix]}.
        naive / weight / hits do not depend on the offsets, so they are formed and
        copied to pinned host memory on a copy stream while the CG runs; only the
        destriped map is copied after the solve (bench.py's chain: 0.73 ms of map copy
        -> ~0.2 ms)."""
        torch = self.torch
        nb, npix, nbo = self.nb, self.npix, self.n_bands
        cur = torch.cuda.current_stream(self.dev)
        m = N.device_empty((4, npix * nb), torch.float64, self.dev)              # map, naive, weight, hits
        nn = self.empty(npix * nb)                                              # local_maps copies it in full
        self._c('comap_destripe_local_maps', self.h, N.dptr(m[2]), N.dptr(m[3]), N.dptr(nn))
        self._c('comap_destripe_div_map', self.h, N.dptr(nn), None, N.dptr(m[1]))
        bands = m.view(4, npix, nb).permute(0, 2, 1)[:, :nbo]                    # [4, n_bands, npix] view
        # unmap: the caller's pixel order from the problem's internal (tiled) one
        static = bands[1:].contiguous() if unmap is None else bands[1:].index_select(2, unmap)
        # page-locked result block from the library's host cache (torch's pinned
        # allocator paid a fresh ~2.5 ms hipHostMalloc on every other solve, r03s7)
        host_np = N.host_empty((4, nbo, npix if unmap is None else int(unmap.numel())))
        host = torch.from_numpy(host_np)
        ready = torch.cuda.Event()
        ready.record(cur)
        cs = copy_stream(self.dev)
        cs.wait_event(ready)
        with torch.cuda.stream(cs):
            host[1:].copy_(static, non_blocking=True)
        static.record_stream(cs)
        x = self.empty(self.n_offsets * nb)                                     # written in full by the solve
        it = (ctypes.c_int32 * nb)()
        self._c('comap_destripe_solve', self.h, float(threshold), int(niter), N.dptr(x), N.dptr(m[0]), None, None,
                None, ctypes.cast(it, ctypes.POINTER(ctypes.c_int32)))
        host[0].copy_(bands[0] if unmap is None else bands[0].index_select(1, unmap), non_blocking=True)
        cur.synchronize()
        cs.synchronize()
        maps = {k: host_np[i] for i, k in enumerate(('map', 'naive', 'weight', 'hits'))}
        return x, [int(v) for v in it][:nbo], maps


_COPY_STREAMS = {}


def copy_stream(dev):
    """One side stream per device for the maps' device -> host copies, kept for the
    process: a torch.cuda.Stream created per problem cost the chain ~1 ms of idle GPU before
    its first CG kernel (the creation waits for the device, r04l trace)."""
    import torch
    key = torch.device(dev).index if not isinstance(dev, int) else dev
    cs = _COPY_STREAMS.get(key)
    if cs is None:
        cs = _COPY_STREAMS[key] = torch.cuda.Stream(dev)
    return cs


TILE = 8     # map layout tile (pixels per side) for a known map shape; COMAP_DS_TILE=0: row-major


_LAYOUTS = {}


def tiled_layout(ny, nx, T, device):
    """Internal id of every row-major pixel of an ny x nx map on a 2-D tiled layout: T x T
    tiles in row-major tile order, the pixels of a tile in Morton (Z) order; and the padded
    internal map size.  The operator then gathers 2-D neighbourhoods from shared cache lines
    and the set-up's spatial offset order (first pixel id) clusters offsets by tile (C5, 8
    obs: 1 band 0.139 -> 0.124, 4 bands 0.295 -> 0.275 ms per CG iteration with T = 8,
    scripts/ds_tiling_probe.py, profiles/r05/r05c_py2.log)."""
    import torch
    if T < 1 or T & (T - 1):
        raise ValueError(f'tile size must be a power of two, not {T}')
    key = (int(ny), int(nx), int(T), str(device))
    if key in _LAYOUTS:
        return _LAYOUTS[key]
    p = torch.arange(ny * nx, device=device, dtype=torch.int64)
    y, x = p // nx, p % nx
    ntx, nty = (nx + T - 1) // T, (ny + T - 1) // T
    ix, iy = x % T, y % T
    z = torch.zeros_like(p)
    for b in range(max(1, (T - 1).bit_length())):
        z |= ((ix >> b) & 1) << (2 * b)
        z |= ((iy >> b) & 1) << (2 * b + 1)
    ids = (((y // T) * ntx + x // T) * T * T + z).to(torch.int32)
    _LAYOUTS[key] = (ids, ntx * nty * T * T)
    return _LAYOUTS[key]


class DeviceDestriper:
    """Convenience wrapper: the whole destriper_iteration on device tensors.

    One band ([N] tod/weights): solve() -> {'x': [N/L], 'iters': int,
    'maps': {k: [npix]}}.  Several bands ([n_bands, N], one batched system):
    {'x': [n_bands, N/L], 'iters': [per band], 'maps': {k: [n_bands, npix]}}.

    Across ranks (torch.distributed initialised, world > 1) every rank passes its own
    samples and gets its own offsets and the full maps.  The problem is either
    sharded (each rank's operator, RCCL all-reduces every CG iteration) or gathered
    to rank 0, which solves it alone and hands back each rank's offsets and the maps:
    mapmaking/rankplan.py models both (COMAP_DS_RANKS=auto: small problems such as one
    observation (C4) are latency-bound across ranks and are gathered, large ones (C5)
    sharded).  The default is COMAP_DS_RANKS=shard until a multi-GPU run replaces the
    model's assumed all-reduce latency and bandwidth; gather forces the other."""

    def __init__(self, pixels, tod, weights, offset_length, npix, device=None, keep=None, map_shape=None):
        """map_shape (ny, nx): the map's row-major layout (CAR / WCS maps), when known; the
        operator then runs on a 2-D tiled internal pixel order (tiled_layout) and the maps
        come back in the caller's order."""
        self.layout, self.okey = None, None
        T = int(os.environ.get('COMAP_DS_TILE', str(TILE)))
        if T > 0 and T & (T - 1):
            # the Morton code inside a tile interleaves log2(T) bits: for another T it would
            # exceed T * T - 1 and merge distinct pixels of neighbouring tiles
            raise ValueError(f'COMAP_DS_TILE must be 0 (row-major) or a power of two, not {T}')
        if map_shape is not None and T > 0:
            ny, nx = (int(v) for v in map_shape)
            if ny * nx != int(npix):
                raise ValueError(f'map_shape {map_shape} does not hold {npix} pixels')
            pixels, npix = self._tile(pixels, int(npix), ny, nx, T, device, int(offset_length))
        self.npix_full, self.hit_index = int(npix), None
        self.multi = np.ndim(tod) == 2 if not hasattr(tod, 'dim') else tod.dim() == 2
        self.gathered, self.plan = None, None
        d = _dist()
        if d is not None and d.get_world_size() > 1:
            if self._choose_gather(d, pixels, tod, offset_length):
                self._gather(d, pixels, tod, weights, keep, offset_length, npix, device)
                return
            if os.environ.get('COMAP_DS_COMPACT', '1') != '0':
                pixels, npix = self._compact(pixels, int(npix), device)
        self.ops = N.retry_oom(DeviceOps, pixels, tod, weights, offset_length, npix, device, keep, self.okey)

    # ---- rank policy
    def _choose_gather(self, d, pixels, tod, offset_length):
        import torch
        from . import rankplan
        # default 'shard': the rank model's all-reduce latency / ring bandwidth are assumptions
        # until a multi-GPU run measures them (rankplan.py), so 'auto' is opt-in
        policy = os.environ.get('COMAP_DS_RANKS', 'shard')
        if policy == 'shard':
            return False
        n_local = int(pixels.numel()) if hasattr(pixels, 'numel') else int(np.size(pixels))
        n_bands = (int(tod.shape[0]) if self.multi else 1)
        dev = self._comm_device(d)
        cnt = torch.tensor([n_local], dtype=torch.int64, device=dev)
        parts = [torch.zeros_like(cnt) for _ in range(d.get_world_size())]
        d.all_gather(parts, cnt)
        self.counts = [int(c.item()) for c in parts]
        if policy == 'gather':
            return True
        self.plan = rankplan.plan(sum(self.counts), n_bands, d.get_world_size())
        return self.plan['mode'] == 'gather'

    @staticmethod
    def _comm_device(d):
        import torch
        return torch.device('cuda', torch.cuda.current_device()) if d.get_backend() == 'nccl' else torch.device('cpu')

    def _gather(self, d, pixels, tod, weights, keep, offset_length, npix, device):
        """Inputs of every rank to rank 0 (padded to the largest rank, in rank order);
        rank 0 builds the single-rank operator on their concatenation."""
        import torch
        L = int(offset_length)
        rank, world = d.get_rank(), d.get_world_size()
        cdev = self._comm_device(d)
        nbands = int(tod.shape[0]) if self.multi else 1
        nmax = max(self.counts)

        def as_t(a, dt):
            t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
            return t.to(device=cdev, dtype=dt)

        def gather(t, width):       # t [rows, n_local] -> root: list of [rows, width]
            pad = torch.zeros((t.shape[0], width), dtype=t.dtype, device=cdev)
            pad[:, :t.shape[1]] = t
            parts = [torch.zeros_like(pad) for _ in range(world)] if rank == 0 else None
            d.gather(pad, gather_list=parts, dst=0)
            return parts

        pix = gather(as_t(pixels, torch.int32).reshape(1, -1), nmax)
        td = gather(as_t(tod, torch.float64).reshape(nbands, -1), nmax)
        wd = gather(as_t(weights, torch.float64).reshape(nbands, -1), nmax)
        kp = None
        if keep is not None:
            kp = gather(as_t(keep, torch.uint8).reshape(nbands, -1), nmax // L)
        self.gathered = {'counts': self.counts, 'L': L}
        if rank != 0:
            self.ops = None
            self._ref = (device, nbands)
            return
        dev = torch.device('cuda', N.current_device() if device is None else int(device))
        cat = lambda parts, per: torch.cat([parts[r][:, :c // per] for r, c in enumerate(self.counts)], dim=1).to(dev)  # noqa: E731
        p_all, t_all, w_all = cat(pix, 1).reshape(-1), cat(td, 1), cat(wd, 1)
        k_all = cat(kp, L) if kp is not None else None
        if not self.multi:
            t_all, w_all = t_all.reshape(-1), w_all.reshape(-1)
        self.ops = DeviceOps(p_all, t_all, w_all, L, npix, device, k_all)
        self._ref = (device, nbands)

    def _solve_gathered(self, d, threshold, niter):
        """Rank 0 solves; iterations and maps are broadcast, each rank's offsets sent back."""
        import torch
        rank, world = d.get_rank(), d.get_world_size()
        cdev = self._comm_device(d)
        device, nbands = self._ref
        nb = 4 if nbands == 3 else nbands
        L, counts = self.gathered['L'], self.gathered['counts']
        npix = self.npix_full
        dev = torch.device('cuda', N.current_device() if device is None else int(device))
        nomax = max(counts) // L
        keys = ('map', 'naive', 'weight', 'hits')
        if rank == 0:
            x, it, maps = self.ops.solve_native(threshold, niter)
            its = torch.tensor(list(it) + [0] * (4 - len(it)), dtype=torch.int64, device=cdev)
            mp = torch.stack([maps[k] for k in keys]).to(cdev)
            xv = x.reshape(-1, nb)
            parts, o = [], 0
            for c in counts:
                pad = torch.zeros((nomax, nb), dtype=torch.float64, device=cdev)
                pad[:c // L] = xv[o:o + c // L]
                parts.append(pad)
                o += c // L
        else:
            its = torch.zeros(4, dtype=torch.int64, device=cdev)
            mp = torch.zeros((4, npix * nb), dtype=torch.float64, device=cdev)
            parts = None
        d.broadcast(its, src=0)
        d.broadcast(mp, src=0)
        mine = torch.zeros((nomax, nb), dtype=torch.float64, device=cdev)
        d.scatter(mine, scatter_list=parts, src=0)
        x = mine[:counts[rank] // L].reshape(-1).to(dev)
        it = [int(v) for v in its.cpu()][:nbands]
        maps = {k: mp[i].to(dev) for i, k in enumerate(keys)}
        return x, it, maps, nb, nbands

    def _tile(self, pixels, npix, ny, nx, T, device, L):
        """Relabel the pixel ids onto tiled_layout; a negative id p (an unbinned sample that
        reads m[npix + p]) becomes the negative id that reads the same pixel there.  With
        COMAP_DS_OKEY=centroid (default) the offsets are also ordered by their centroid
        pixel's internal id (comap_offset_centroid_keys) instead of their first pixel: the
        offsets crossing one pixel then sit close together, which is what the CG bin's x
        gathers touch."""
        import torch
        dev = torch.device('cuda', N.current_device() if device is None else int(device))
        pix = pixels.to(device=dev, dtype=torch.int32).reshape(-1) if isinstance(pixels, torch.Tensor) else \
            torch.from_numpy(np.ascontiguousarray(pixels, dtype=np.int32)).to(dev).reshape(-1)
        ids, nt = tiled_layout(ny, nx, T, dev)
        # one device pass (comap_relabel_pixels), no host sync: an id outside [-npix, npix)
        # becomes nt, which the set-up's device range check rejects (IndexError), as it
        # would the original id
        out = torch.empty_like(pix)
        c = N.ctx(dev.index)
        N.bind_stream(c, dev)
        N.check(N.lib().comap_relabel_pixels_tiled(c, N.dptr(pix), pix.numel(), int(nx), int(ny), int(T),
                                                   N.dptr(out)), c, 'comap_relabel_pixels_tiled')
        if os.environ.get('COMAP_DS_OKEY', 'centroid') == 'centroid' and pix.numel() % L == 0:
            keys = torch.empty(pix.numel() // L, dtype=torch.int32, device=dev)
            N.check(N.lib().comap_offset_centroid_keys(c, N.dptr(pix), pix.numel(), int(L), int(nx), int(ny),
                                                       N.dptr(ids), int(nt), N.dptr(keys)), c,
                    'comap_offset_centroid_keys')
            self.okey = (keys, int(nt) + 1)
        self.layout = ids
        return out, nt

    def _untile(self, v, nb):
        """[npix_internal * nb] interleaved map -> the caller's row-major [npix * nb]."""
        if self.layout is None:
            return v
        return v.reshape(-1, nb).index_select(0, self.layout).reshape(-1)   # (int32 ids)

    def _compact(self, pixels, npix, device):
        """Across ranks the map numerator is all-reduced every CG iteration
        (Destriper.py:183-204); only pixels some rank's samples hit can be non-zero.
        Relabel the pixels onto that union, in increasing pixel order, so every
        all-reduce carries the hit pixels only ("compact to hit pixels").
        The relabelling is monotone, and the pixels that unbinned samples read are kept
        (a negative id p reads m[npix + p], Destriper.py:206-213): the per-pixel sums, the
        offsets' spatial order and hence every iterate are unchanged, bit for bit.  Maps are
        expanded back to npix in solve()."""
        import torch
        dev = torch.device('cuda', N.current_device() if device is None else int(device))
        pix = pixels.to(device=dev, dtype=torch.int64).reshape(-1) if isinstance(pixels, torch.Tensor) else \
            torch.from_numpy(np.ascontiguousarray(pixels, dtype=np.int64)).to(dev).reshape(-1)
        if pix.numel() and (int(pix.max().item()) >= npix or int(pix.min().item()) < -npix):
            raise IndexError(f'pixel index out of range for a map of {npix} pixels (valid: -{npix} .. {npix - 1})')
        comp, self.hit_index = compact_pixels(pix, npix, torch_allreduce)
        return comp, int(self.hit_index.numel())

    def _expand(self, v):
        """[n_hit * nb] interleaved map on the compacted pixels -> [npix * nb]."""
        if self.hit_index is None:
            return v
        nb = self.ops.nb
        out = self.ops.torch.zeros((self.npix_full, nb), dtype=v.dtype, device=v.device)
        out[self.hit_index] = v.reshape(-1, nb)
        return out.reshape(-1)

    def nnz(self):
        return self.ops.nnz()

    def entry_bytes(self):
        return self.ops.entry_bytes()

    def sell_entries(self):
        return self.ops.sell_entries()

    def solve(self, threshold=1e-6, niter=100, to_host=False, allreduce=None):
        """to_host: maps as host NumPy arrays (rank 0; None on the others) -- one
        rank solving alone overlaps their copy with the CG (solve_native_host).
        allreduce: the sharded CG's sum across ranks (default torch_allreduce; bench.py
        passes a TimedAllreduce to measure the per-iteration collective cost)."""
        d = _dist()
        ops = self.ops
        if to_host and self.gathered is None and (d is None or d.get_world_size() == 1):
            x, it, maps = ops.solve_native_host(threshold, niter, unmap=self.layout)
            maps['map2'] = maps['weight']
            if not self.multi:
                return {'x': x, 'iters': it[0], 'maps': {k: v[0] for k, v in maps.items()}}
            return {'x': ops.split_bands(x), 'iters': it, 'maps': maps}
        if to_host:
            res = self.solve(threshold, niter)
            rank = d.get_rank() if d is not None else 0
            res['maps'] = maps_to_host(res['maps']) if rank == 0 else None
            return res
        if self.gathered is not None:
            x, it, maps, nb, nbands = self._solve_gathered(d, threshold, niter)
            split = lambda v: v.reshape(-1, nb).t()[:nbands].contiguous()   # noqa: E731
        elif d is None or d.get_world_size() == 1:
            x, it, maps = ops.solve_native(threshold, niter)
            split = ops.split_bands
        else:
            # COMAP_DS_GRAPH=1: the captured-graph driver (one launch per 16 iterations);
            # default: the eager batched driver (7 host calls per iteration, 16 per check)
            # (graph capture of a collective needs RCCL: with any other backend, e.g. the gloo
            # rehearsals, the eager driver runs instead)
            solver = cg_solve_batched
            if os.environ.get('COMAP_DS_GRAPH') == '1':
                if d.get_backend() == 'nccl':
                    solver = cg_solve_graph
                else:
                    import warnings
                    warnings.warn(f'COMAP_DS_GRAPH=1 needs the nccl (RCCL) backend, not {d.get_backend()}: '
                                  'using the eager CG driver')
            x, it, h, nnum = solver(ops, allreduce or torch_allreduce, threshold, niter)
            _, hits, _ = ops.local_maps()
            torch_allreduce(hits)
            num = ops.zeros(ops.npix * ops.nb)
            ops.bin(x, 1, num)
            torch_allreduce(num)
            maps = {'map': ops.zeros(ops.npix * ops.nb), 'naive': ops.zeros(ops.npix * ops.nb), 'weight': h,
                    'hits': hits}
            ops.div_map(num, h, maps['map'])
            ops.div_map(nnum, h, maps['naive'])
            it = it[:ops.n_bands]
            x = ops.natural(x)
            maps = {k: self._expand(v) for k, v in maps.items()}
            split = ops.split_bands
        if self.layout is not None:
            nbl = nb if self.gathered is not None else ops.nb
            maps = {k: self._untile(v, nbl) for k, v in maps.items()}
        if not self.multi:
            maps['map2'] = maps['weight']
            return {'x': x, 'iters': it[0], 'maps': maps}
        maps = {k: split(v) for k, v in maps.items()}
        maps['map2'] = maps['weight']
        return {'x': split(x), 'iters': it, 'maps': maps}


def maps_to_host(maps):
    """{name: device tensor} -> {name: NumPy array}: one device-side stack and one copy
    into page-locked host memory from the library's cache (a pageable copy per map runs
    at a fraction of the link)."""
    import torch
    keys = list(maps)
    if not keys:
        return {}
    flat = torch.stack([maps[k].reshape(-1) for k in keys])
    a = N.host_empty(tuple(flat.shape), str(flat.dtype).split('.')[-1])    # cached page-locked block
    torch.from_numpy(a).copy_(flat, non_blocking=True)
    torch.cuda.current_stream(flat.device).synchronize()
    return {k: a[i].reshape(tuple(maps[k].shape)) for i, k in enumerate(keys)}


def run_destriper(_pointing, _tod, _weights, offset_length, pixel_edges, az=None, el=None, ra=None, dec=None,
                  feedid=None, obsids=None, obsid_cuts=None, threshold=1e-6, niter=100, chi2_cutoff=100,
                  special_weight=None, healpix=False, device=None, map_shape=None):
    """Destriper.run_destriper (Destriper.py:456-503) on the GPU.

    ``pixel_edges[-1] + 1`` is the map size (bin_offset_map, :169).  Returns
    {'All': maps} with host NumPy maps on rank 0; other ranks get None maps.
    map_shape (ny, nx), an extension: the map's row-major layout, which lets the
    operator run on a 2-D tiled pixel order (DeviceDestriper)."""
    if special_weight is not None:
        raise NotImplementedError('special_weight is unused by run_destriper in the reference (:482)')
    import torch
    if device is None:
        device = torch.cuda.current_device()
    npix = int(pixel_edges[-1]) + 1
    dd = DeviceDestriper(np.asarray(_pointing), np.asarray(_tod, dtype=np.float64),
                         np.asarray(_weights, dtype=np.float64), int(offset_length), npix, device, map_shape=map_shape)
    res = dd.solve(threshold, niter, to_host=True)
    d = _dist()
    rank = d.get_rank() if d is not None else 0
    if rank != 0:
        return {'All': {'map': None, 'naive': None, 'weight': None, 'map2': None}}
    return {'All': res['maps']}


def run_destriper_bands(_pointing, _tods, _weights, offset_length, pixel_edges, keep=None, threshold=1e-6,
                        niter=100, device=None, map_shape=None):
    """run_destriper for several sidebands on the same pointing in ONE batched
    device solve (the reference calls run_destriper once per band,
    run_destriper.py:146-189).  _tods/_weights [n_bands, N]; keep [n_bands, N/L]
    as returned by comapdata.read_comap_data_bands.  Returns one
    {'All': maps} per band (host maps on rank 0, None maps on other ranks);
    band b's maps and iteration count are those of run_destriper on band b's
    own samples, and its offsets (``x``, rank 0: also under 'offsets') cover
    the union of the bands' offsets (0 where band b dropped the offset)."""
    import torch
    if device is None:
        device = torch.cuda.current_device()
    npix = int(pixel_edges[-1]) + 1
    tods = np.asarray(_tods, dtype=np.float64)
    if tods.ndim != 2:
        raise ValueError('_tods must be [n_bands, N]')
    dd = DeviceDestriper(np.asarray(_pointing), tods, np.asarray(_weights, dtype=np.float64), int(offset_length), npix,
                         device, keep=None if keep is None else np.asarray(keep, dtype=np.uint8), map_shape=map_shape)
    res = dd.solve(threshold, niter, to_host=True)
    d = _dist()
    rank = d.get_rank() if d is not None else 0
    out = []
    hm = res['maps']
    for b in range(tods.shape[0]):
        if rank != 0:
            out.append({'All': {'map': None, 'naive': None, 'weight': None, 'map2': None}})
            continue
        maps = {k: v[b] for k, v in hm.items()}
        out.append({'All': maps, 'iters': res['iters'][b], 'offsets': res['x'][b].cpu().numpy()})
    return out


# ---------------------------------------------------------------- bench helper
def car_pixels(ra, dec, nx=480, ny=480, cdelt=1.0 / 60.0, ra0=None, dec0=None):
    """Plate-carree pixel index (floor(x + 0.5) convention of transform_to_1d,
    COMAPData.py:83-117) of (ra, dec) on an nx x ny grid centred on (ra0, dec0);
    off-map -> -1.  A fp64 restatement of CAR without wcslib (WCS parity is
    SURVEY §8f row 1)."""
    import torch
    ra0 = float(torch.median(ra)) if ra0 is None else ra0
    dec0 = float(torch.median(dec)) if dec0 is None else dec0
    px = torch.floor(-(ra - ra0) / cdelt + (nx / 2 - 1) + 0.5)
    py = torch.floor((dec - dec0) / cdelt + (ny / 2 - 1) + 0.5)
    ok = (px >= 0) & (px <= nx - 1) & (py >= 0) & (py <= ny - 1)
    return torch.where(ok, py * nx + px, torch.full_like(px, -1)).to(torch.int32)


def level2_to_destriper_inputs(level2, data, band=0, offset_length=50):
    """Flat (tod, weights, pixels) device tensors from a Level-2 result: per
    feed and scan the first floor(n/L)*L samples (countDataSize,
    COMAPData.py:163-187), weights = averaged_tod/weights.  The cuts and the
    w=400 median filter of get_tod are SURVEY §8f row 1 (not applied here)."""
    import torch
    tod = level2['averaged_tod/tod']
    w = level2['averaged_tod/weights']
    dev = tod.device
    ra = torch.as_tensor(np.asarray(data['spectrometer/pixel_pointing/pixel_ra']), device=dev)
    dec = torch.as_tensor(np.asarray(data['spectrometer/pixel_pointing/pixel_dec']), device=dev)
    edges = np.asarray(level2['averaged_tod/scan_edges'])
    segs_t, segs_w, segs_p = [], [], []
    ra0, dec0 = float(torch.median(ra)), float(torch.median(dec))
    for f in range(tod.shape[0]):
        for s, e in edges:
            n = int((e - s) // offset_length * offset_length)
            if n <= 0:
                continue
            segs_t.append(tod[f, band, s:s + n])
            segs_w.append(w[f, band, s:s + n])
            segs_p.append(car_pixels(ra[f, s:s + n], dec[f, s:s + n], ra0=ra0, dec0=dec0))
    t = torch.cat(segs_t)
    ww = torch.cat(segs_w)
    pp = torch.cat(segs_p)
    bad = ~torch.isfinite(t)
    t = torch.where(bad, torch.zeros_like(t), t)
    ww = torch.where(bad | ~torch.isfinite(ww), torch.zeros_like(ww), ww)
    return t, ww, pp
