"""One observation's L1 -> L2 reduction sharded over ranks (BASELINE configs[2], C3).

The reference parallelises over whole files (run_average.py:38-39: contiguous
blocks of the file list per MPI rank).  One 19-feed observation is the unit of
work here, so it is split by its (feed, scan) units instead -- SURVEY.md §8(e):
every step of Level1AveragingGainCorrection.average_tod (Level1Averaging.py:
792-872) is independent per (feed, scan), the gain solve couples only the 4
bands x 1024 channels of one unit, and the vane calibration
(VaneCalibration.py:143-198) is per feed.  So each rank

  * takes a contiguous run of units (feed-major order, balanced by samples),
  * holds only the feeds its units touch (a feed split between two ranks is
    held by both; its vane is computed by both, identically),
  * reduces them with no collective, and
  * owns the output slices of its units: averaged_tod[f, :, t0:t0+n] and
    atmosphere/fit_values[s, f].

``assemble`` rebuilds the full-observation Level-2 arrays from the shards'
outputs (outside the reduction; the tests use it to show that 1 and N shards
give bit-identical results).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .datahandling import COMAPLevel1, to_host

# datasets with a leading feed axis (sliced per shard)
FEED_AXIS_PATHS = ('spectrometer/tod', 'spectrometer/band_average', 'spectrometer/feeds',
                   'spectrometer/pixel_pointing/pixel_ra', 'spectrometer/pixel_pointing/pixel_dec',
                   'spectrometer/pixel_pointing/pixel_az', 'spectrometer/pixel_pointing/pixel_el')


def unit_table(edges, n_feeds: int) -> np.ndarray:
    """All (feed index, scan index, first sample, n samples) units with n > 0, in the
    order the device plan uses (feed-major, scans ascending)."""
    edges = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    rows = [(f, s, int(a), int(b - a)) for f in range(n_feeds) for s, (a, b) in enumerate(edges) if b > a]
    return np.array(rows, dtype=np.int64).reshape(-1, 4)


def partition_units(weights, world: int) -> list:
    """Contiguous split of units with the given weights (samples) into ``world``
    runs minimising the largest run (binary search on the bound + greedy fill).
    Returns [(lo, hi)] unit index ranges, one per rank (a rank may get none)."""
    w = np.asarray(weights, dtype=np.int64)
    n = w.size
    if world < 1:
        raise ValueError('world must be >= 1')

    def runs(bound):
        out, lo, acc = [], 0, 0
        for i in range(n):
            if acc + w[i] > bound and i > lo:
                out.append((lo, i))
                lo, acc = i, 0
            acc += w[i]
        out.append((lo, n))
        return out

    if n == 0:
        return [(0, 0)] * world
    lo_b, hi_b = int(w.max()), int(w.sum())
    while lo_b < hi_b:
        mid = (lo_b + hi_b) // 2
        if len(runs(mid)) <= world:
            hi_b = mid
        else:
            lo_b = mid + 1
    r = runs(lo_b)
    r += [(n, n)] * (world - len(r))
    return r


@dataclass
class Shard:
    rank: int
    world: int
    units: np.ndarray          # [k, 4] global (feed, scan, t0, n) of this rank
    f_lo: int                  # feeds [f_lo, f_hi) held by this rank
    f_hi: int

    @property
    def n_feeds(self) -> int:
        return self.f_hi - self.f_lo

    def local_filter(self) -> np.ndarray:
        """(feed index within the shard, scan index) of the owned units."""
        u = self.units
        return np.stack([u[:, 0] - self.f_lo, u[:, 1]], axis=1) if u.size else np.zeros((0, 2), np.int64)

    def samples_x_channels(self) -> int:
        return int(self.units[:, 3].sum()) * 4 * 1024 if self.units.size else 0


def shard_for(edges, n_feeds: int, rank: int, world: int) -> Shard:
    units = unit_table(edges, n_feeds)
    lo, hi = partition_units(units[:, 3], world)[rank]
    mine = units[lo:hi]
    if mine.size == 0:
        return Shard(rank, world, mine, 0, 0)
    return Shard(rank, world, mine, int(mine[:, 0].min()), int(mine[:, 0].max()) + 1)


def slice_feeds(data: COMAPLevel1, f_lo: int, f_hi: int, unit_filter=None) -> COMAPLevel1:
    """A COMAPLevel1 holding feeds [f_lo, f_hi) of ``data`` (views where possible;
    datasets without a feed axis are shared).  ``unit_filter`` [k, 2] (feed index
    within the slice, scan) restricts the device reduction to those units."""
    out = COMAPLevel1(overwrite=data.overwrite, large_datasets=list(data.large_datasets))
    for k, v in data.items():
        if k in FEED_AXIS_PATHS:
            out[k] = v.rows(f_lo, f_hi) if hasattr(v, 'rows') else v[f_lo:f_hi]   # file-backed: stays lazy
        else:
            out[k] = v
    for p, a in data.items(attr=True):
        for k, v in a.items():
            out.set_attrs(p, k, v)
    if unit_filter is not None:
        out.unit_filter = np.asarray(unit_filter, dtype=np.int64).reshape(-1, 2)
    return out


def shard_level1(data: COMAPLevel1, rank: int, world: int):
    """(Shard, the rank's COMAPLevel1) for a full observation held on the host."""
    edges = np.asarray(to_host(data.scan_edges), dtype=np.int64).reshape(-1, 2)
    F = int(np.asarray(to_host(data['spectrometer/feeds'])).size)
    sh = shard_for(edges, F, rank, world)
    return sh, slice_feeds(data, sh.f_lo, sh.f_hi, sh.local_filter())


def assemble(shards, outputs, n_feeds: int, n_scans: int, n_samples: int) -> dict:
    """Full-observation Level-2 arrays from per-shard results.

    outputs[i] (shard i): {'averaged_tod/tod'|'tod_original'|'weights': [Fi, 4, T],
    'atmosphere/fit_values': [S, Fi, 4, 2, 1024], 'vane/system_temperature'|
    'vane/system_gain': [nV, Fi, 4, 1024]} (host or device arrays).  Each unit's
    slice is taken from the shard that owns it; a feed held by several shards
    takes its vane from the first."""
    T = n_samples
    full = {k: np.zeros((n_feeds, 4, T)) for k in ('averaged_tod/tod', 'averaged_tod/tod_original',
                                                  'averaged_tod/weights')}
    full['atmosphere/fit_values'] = np.full((n_scans, n_feeds, 4, 2, 1024), np.nan)
    vane_done = np.zeros(n_feeds, dtype=bool)
    for sh, out in zip(shards, outputs):
        if sh.units.size == 0:
            continue
        host = {k: to_host(v) for k, v in out.items()}
        for f, s, t0, n in sh.units:
            fl = f - sh.f_lo
            for k in ('averaged_tod/tod', 'averaged_tod/tod_original', 'averaged_tod/weights'):
                full[k][f, :, t0:t0 + n] = host[k][fl, :, t0:t0 + n]
            full['atmosphere/fit_values'][s, f] = host['atmosphere/fit_values'][s, fl]
        new = [f for f in range(sh.f_lo, sh.f_hi) if not vane_done[f]]
        for k in ('vane/system_temperature', 'vane/system_gain'):
            if k not in host:
                continue
            if k not in full:
                full[k] = np.zeros((host[k].shape[0], n_feeds) + host[k].shape[2:])
            for f in new:
                full[k][:, f] = host[k][:, f - sh.f_lo]
        vane_done[sh.f_lo:sh.f_hi] = True
    return full
