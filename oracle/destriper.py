"""ORACLE (test infrastructure only): the destriper restated in NumPy.

Follows comancpipeline/MapMaking/Destriper.py (v0.9.1):
  bin_offset_map  :155-181   two binValues passes (sum z w, sum w)
  share_map       :183-204   sum over ranks, m /= h where h != 0
  op_Z            :206-213   tod - m[pointing]  (pointing -1 wraps to m[-1])
  op_Ax.__call__  :217-263   F^T W Z F, F = repeat(x, L)
  cgm             :85-152    BiCG; p == pb and r == rb bit for bit, so one
                             matvec per iteration reproduces its iterates
  destriper_iteration :402-453  final maps (map, naive, weight, hits)

``ShardOps`` exposes the same operator pieces per rank (local partial map
numerators, local dot products) so tests can drive the product's
distributed CG driver (comapreduce_amd.mapmaking.destriper.cg_solve) on
several CPU ranks with the gloo backend.
"""
import numpy as np

from . import bin_values


def bin_offset_map(pointing, z, w, npix):
    m = np.zeros(npix)
    h = np.zeros(npix)
    bin_values(m, pointing, weights=z * w)
    bin_values(h, pointing, weights=w)
    return m, h


def share_map(m, h):
    m = m.copy()
    nz = h != 0
    m[nz] /= h[nz]
    return m


def op_Ax(x, pointing, w, L, npix, extend=True):
    z = np.repeat(x, L) if extend else x
    m, h = bin_offset_map(pointing, z, w, npix)
    m = share_map(m, h)
    diff = z - m[pointing]
    return np.sum(np.reshape(diff * w, (z.size // L, L)), axis=1)


def cgm(A, b, threshold=1e-6, niter=100):
    """Destriper.py:85-152 with the duplicate matvecs folded (p == pb)."""
    x = np.zeros(b.size)
    r = b - A(x)
    p = r.copy()
    thresh0 = np.sum(r * r)
    it = 0
    for i in range(niter):
        q = A(p)
        rr = np.sum(r * r)
        alpha = rr / np.sum(p * q)
        x += alpha * p
        r = r - alpha * q
        rr_new = np.sum(r * r)
        beta = rr_new / rr
        p = r + beta * p
        it = i + 1
        delta = rr_new / thresh0
        if np.isnan(delta) or delta < threshold:
            break
    return x, it


def destriper_iteration(pointing, tod, w, L, npix, threshold=1e-6, niter=100):
    A = lambda x: op_Ax(x, pointing, w, L, npix)                           # noqa: E731
    b = op_Ax(tod, pointing, w, L, npix, extend=False)
    x, it = cgm(A, b, threshold, niter)
    n, h = bin_offset_map(pointing, tod, w, npix)
    m, _ = bin_offset_map(pointing, tod - np.repeat(x, L), w, npix)
    _, hits = bin_offset_map(pointing, tod, np.ones(tod.size), npix)
    nz = h != 0
    m[nz] /= h[nz]
    n[nz] /= h[nz]
    return {'map': m, 'naive': n, 'weight': h, 'map2': h, 'hits': hits}, x, it


class ShardOps:
    """One rank's share of the samples (whole offsets), NumPy operators with
    the interface of comapreduce_amd.mapmaking.destriper.DeviceOps."""

    def __init__(self, pointing, tod, w, L, npix):
        self.p, self.tod, self.w, self.L, self.npix = pointing, tod, w, L, npix
        self.n_offsets = tod.size // L
        self.h = np.zeros(npix)
        self.hits = np.zeros(npix)
        self.nnum = np.zeros(npix)
        bin_values(self.h, pointing, weights=w)
        bin_values(self.hits, pointing)
        bin_values(self.nnum, pointing, weights=tod * w)

    def zeros(self, n):
        return np.zeros(n)

    def scalar(self):
        return np.zeros(1)

    def copy(self, a):
        return a.copy()

    def local_maps(self):
        return self.h.copy(), self.hits.copy(), self.nnum.copy()

    def bin(self, x, mode, out):
        m = np.zeros(self.npix)
        bin_values(m, self.p, weights=np.repeat(x, self.L) * self.w)
        out[:] = (self.nnum - m) if mode == 1 else m

    def project(self, x, num, h, y, dot=None):
        m = share_map(num, h)
        z = self.tod if x is None else np.repeat(x, self.L)
        y[:] = np.sum(np.reshape((z - m[self.p]) * self.w, (self.n_offsets, self.L)), axis=1)
        if dot is not None:
            dot[0] = np.sum(y * x)

    def dot(self, a, b, out):
        out[0] = np.sum(a * b)

    def cg_update(self, rr, pq, x, r, p, q, rr_new):
        a = rr[0] / pq[0]
        x += a * p
        r -= a * q
        rr_new[0] = np.sum(r * r)

    def cg_direction(self, rr_new, rr, p, r):
        p[:] = r + (rr_new[0] / rr[0]) * p

    def div_map(self, num, h, out):
        out[:] = share_map(num, h)

    def host_scalar(self, s):
        return float(s[0])

    def set_scalar(self, dst, src):
        dst[0] = src[0]
