"""Destriper data prep: Level-2 files -> flat (tod, weights, pointing, ...) vectors.

Mirror of reference comancpipeline/MapMaking/COMAPData.py (same function
names, arguments and outputs).  ``read_comap_data`` / ``read_comap_data_bands``
run on the GPU (mapmaking/prep.py -> csrc/prep_kernels.hip): per file one
launch each for the weights (auto_rms), the az / el percentiles and the
per-sample gather (cuts, Sun distance, pixel ids), one batched 400-sample
high-pass for the rank, one cut + compaction.  The host handles per-file
metadata only.  There is no CPU fallback.

Reference behaviours kept on purpose:
  * weights = 1/auto_rms(tod)^2 with auto_rms's ``tod[:-1:N]`` slicing bug
    (= nanstd(tod[1:N] - tod[0]) / sqrt 2) over the whole file TOD;
  * spike mask, Sun "distance" < 10 deg (healpy inverse rotation +
    haversine of (phi, theta) -- COMAPData.py:213-236, 326-327), az/el
    outside the 10-90th percentiles and the first/last 10% of each scan get
    weight 0; feeds whose bad_observation bits include anything but 0 and 5
    are skipped;
  * read_pixels fills row ``ifeed`` from row ``output_feed`` of the file
    pointing (COMAPData.py:423-424);
  * offsets whose weights are all zero are dropped after concatenation.
"""
from __future__ import annotations

import os

import numpy as np

from . import astro
from .wcs import CelestialWCS, transform_to_1d
from ..pipeline.datahandling import HDF5Data

CALIBRATORS = ('TauA', 'CasA', 'CygA', 'jupiter')
MEDFILT_STEP = 400


# --------------------------------------------------------------------- file access
class Level2File:
    """Read-only view of a Level-2 file: ``f[path]`` and ``f.attrs(group)``."""

    def __init__(self, datasets: dict, attrs: dict, filename: str = ''):
        self._d, self._a, self.filename = datasets, attrs, filename

    @classmethod
    def open(cls, filename: str):
        h = HDF5Data(name='Level2')
        path = filename if os.path.exists(filename) else filename + '.npz'
        h.read_data_file(path)
        return cls(dict(h.items()), dict(h.items(attr=True)), filename)

    def __getitem__(self, k):
        return self._d[k]

    def __contains__(self, k):
        return k in self._d

    def attrs(self, group):
        return self._a[group]


def _opener(store):
    if store is None:
        return Level2File.open
    return lambda fn: Level2File(store[fn][0], store[fn][1], fn)


# --------------------------------------------------------------------- helpers
def auto_rms(tod):
    """COMAPData.auto_rms (COMAPData.py:205-208), slicing bug included."""
    N = tod.size // 2 * 2
    diff = tod[1:N] - tod[:-1:N]
    return np.nanstd(diff) / np.sqrt(2)


def parse_bit_mask(flag):
    """COMAPData.parse_bit_mask (COMAPData.py:29-40): set bit positions, highest
    first; the reference loop appends a final 0 unless it stopped on bit 0."""
    flag = int(flag)
    bits = [p for p in range(flag.bit_length() - 1, -1, -1) if flag >> p & 1]
    if not bits or bits[-1] != 0:
        bits.append(0)
    return bits


def feed_is_bad(flag):
    return any(b not in (0, 5) for b in parse_bit_mask(flag))


def GetFeeds(file_feeds, selected_feeds):
    """COMAPData.GetFeeds (COMAPData.py:138-154)."""
    file_feeds = np.asarray(file_feeds)
    sel = np.asarray(selected_feeds)
    fi = np.argmin(np.abs(sel[:, None] - file_feeds[None, :]), axis=1)
    fi = fi[file_feeds[fi] == sel]
    oi = np.argmin(np.abs(file_feeds[:, None] - sel[None, :]), axis=1)
    oi = oi[sel[oi] == file_feeds]
    return fi, oi


def get_scan_edges(f):
    return f['averaged_tod/scan_edges'] if 'averaged_tod/scan_edges' in f else [[0, 0]]


def scan_lengths(edges, offset_length):
    return [int((e - s) // offset_length * offset_length) for s, e in edges]


def countDataSize(f, Nfeeds, offset_length):
    """COMAPData.countDataSize (COMAPData.py:163-187)."""
    N = sum(scan_lengths(get_scan_edges(f), offset_length))
    return {'datasize': N * 1.0, 'N': int(N * Nfeeds)}


def find_unique_values(values, comm=None):
    """COMAPData.find_unique_values (COMAPData.py:60-70): union over ranks."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, np.asarray(values).tolist())
        values = [v for p in parts for v in p]
    return np.unique(values)


def map_info_from(crval, cdelt, crpix, ctype, nxpix, nypix):
    """The map_info dict run_destriper.main builds (run_destriper.py:118-128)."""
    return {'wcs': CelestialWCS(crval, cdelt, crpix, ctype), 'nxpix': int(nxpix), 'nypix': int(nypix)}


# --------------------------------------------------------------------- per file
def read_pixels(f, datasize, offset_length, selected_feeds, map_info):
    """COMAPData.read_pixels (COMAPData.py:383-427), all scans in one transform."""
    fi, oi = GetFeeds(f['spectrometer/feeds'], selected_feeds)
    wcs, nx, ny = map_info['wcs'], map_info['nxpix'], map_info['nypix']
    edges = get_scan_edges(f)
    lens = scan_lengths(edges, offset_length)
    cols = np.concatenate([np.arange(s, s + n) for (s, _), n in zip(edges, lens)]) if lens else np.zeros(0, int)
    x = f['spectrometer/pixel_pointing/pixel_ra'][fi][:, cols]
    y = f['spectrometer/pixel_pointing/pixel_dec'][fi][:, cols]
    if 'GLON' in wcs.ctype[0]:
        gb, gl = astro.Rotator(coord=['C', 'G'])((90 - y.ravel()) * np.pi / 180., x.ravel() * np.pi / 180.)
        x, y = gl * 180. / np.pi, (np.pi / 2 - gb) * 180. / np.pi
    p = transform_to_1d(np.ravel(x), np.ravel(y), wcs, nx, ny).reshape(len(fi), cols.size)
    pixels = np.zeros((len(oi), datasize))
    n = min(len(oi), len(fi))
    pixels[:n, :cols.size] = p[oi[:n]]
    return pixels


def read_pixels_healpix(f, datasize, offset_length, selected_feeds, map_info, nside=4096):
    """COMAPData.read_pixels_healpix (COMAPData.py:429-469): healpy.ang2pix RING
    pixels (nside 4096) of every scan sample (galactic for a GLON map), rows in
    the file's feed order (the reference does not remap them to the output
    order as read_pixels does; with every selected feed present they coincide)."""
    from . import healpix
    fi, oi = GetFeeds(f['spectrometer/feeds'], selected_feeds)
    wcs = map_info['wcs']
    edges = f['averaged_tod/scan_edges']
    lens = scan_lengths(edges, offset_length)
    cols = np.concatenate([np.arange(s, s + n) for (s, _), n in zip(edges, lens)]) if lens else np.zeros(0, int)
    x = f['spectrometer/pixel_pointing/pixel_ra'][fi][:, cols]
    y = f['spectrometer/pixel_pointing/pixel_dec'][fi][:, cols]
    if 'GLON' in wcs.ctype[0]:
        gb, gl = astro.Rotator(coord=['C', 'G'])((90 - y.ravel()) * np.pi / 180., x.ravel() * np.pi / 180.)
        x, y = gl * 180. / np.pi, (np.pi / 2 - gb) * 180. / np.pi
    p = healpix.ang2pix(nside, (90 - np.ravel(y)) * np.pi / 180., np.ravel(x) * np.pi / 180).reshape(len(fi), cols.size)
    pixels = np.zeros((len(oi), datasize))
    n = min(len(oi), len(fi))
    pixels[:n, :cols.size] = p[:n]
    return pixels


def read_comap_data(filelist, map_info, feed_weights=None, iband=0, use_gain_filter=True, offset_length=50,
                    feeds=[i + 1 for i in range(19)], calibration=False, calibrator='TauA', healpix=False,
                    store=None, device=None, device_outputs=False):
    """COMAPData.read_comap_data (COMAPData.py:471-577): same arguments and
    return tuple ``(tod, weights, pointing, remapping_array, az, el, ra, dec,
    feedid, obsids)``, computed on the GPU (mapmaking/prep.py).  ``store``
    (tests, the in-memory chain) maps filename -> (datasets, attrs); ``device``:
    the rank's GPU (default: torch's current device); ``device_outputs``: torch
    CUDA tensors instead of NumPy arrays."""
    r = read_comap_data_bands(filelist, map_info, bands=(iband,), use_gain_filter=use_gain_filter,
                              offset_length=offset_length, feeds=feeds, calibration=calibration,
                              calibrator=calibrator, healpix=healpix, store=store, device=device,
                              device_outputs=device_outputs)
    return (r['tod'][0], r['weights'][0], r['pointing'], r['remapping_array'], r['az'], r['el'], r['ra'], r['dec'],
            r['feedid'], r['obsids'])


def read_comap_data_bands(filelist, map_info, bands=(0, 1, 2, 3), use_gain_filter=True, offset_length=50,
                          feeds=[i + 1 for i in range(19)], calibration=False, calibrator='TauA', healpix=False,
                          store=None, device=None, device_outputs=False, pointing=None):
    """read_comap_data for several bands at once, for the batched destriper
    (run_destriper.py:146-189 calls read_comap_data once per band on the same
    files; only tod and weights depend on the band).  One device prep for all
    bands (mapmaking/prep.py: get_tod / read_pixels on the GPU, one batched
    400-sample high-pass, one cut).

    Each band gets the reference's NaN cut (tod and weight 0).  The reference
    then drops the offsets whose weights are all zero -- per band, so the
    bands' sample sets differ; here the samples of every offset that ANY band
    keeps are returned, with keep[b, o] saying whether band b's own
    read_comap_data would have kept offset o (its weights there are all 0 when
    not).  Band b's kept samples, in order, are exactly what
    read_comap_data(iband=b) returns.

    Returns dict: tod, weights [nb, N]; keep uint8 [nb, N/L]; pointing, az, el,
    ra, dec, feedid, obsids [N]; remapping_array (unique pixels of the union).
    NumPy arrays, or torch CUDA tensors with device_outputs (remapping_array
    stays NumPy).  ``pointing``: prep.precompute_pointing's result for these files
    (the az / el percentiles computed ahead, e.g. beside the Level-1 reduction)."""
    import torch
    from . import prep
    open_file = _opener(store)
    bands = tuple(int(b) for b in bands)
    files = [open_file(fn) for fn in filelist]
    flat = prep.prep_flat(files, filelist, map_info, bands, use_gain_filter, offset_length, feeds, calibration,
                          calibrator, device, healpix, pointing)
    cut, keep = prep.cut_flat(flat, len(bands), offset_length)
    del flat
    mark = prep._Phases(torch, cut.tod.device)
    pointing = cut.pix.to(torch.int64)
    if healpix:
        local = torch.unique(pointing)
    else:   # map pixels (and -1) are bounded by the map: a hit mask, no sort
        hit = torch.zeros(int(map_info['nxpix']) * int(map_info['nypix']) + 1, dtype=torch.uint8,
                          device=pointing.device)
        hit[pointing + 1] = 1
        local = torch.nonzero(hit).reshape(-1) - 1
    import torch.distributed as dist
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if healpix or multi or not device_outputs:
        # the union over ranks is a collective: every rank forms it here, in call order
        remapping_array = find_unique_values(local.cpu().numpy()).astype(int)
    else:
        # one rank, device outputs (the in-memory chain): the union is the local set; it is
        # copied to the host only when read, so the prep queues on without a host round trip
        remapping_array = None
    mark('unique')
    if healpix:      # COMAPData.py:572-573: pixel ids -> positions in the union over ranks
        # index_replace (COMAPData.py:43-58) as written: the inverse sort permutation
        # indexed by the searchsorted positions (the identity for np.unique's sorted union)
        order = np.argsort(remapping_array)
        inv = np.empty_like(order)
        inv[order] = np.arange(order.size)
        ra_sorted = torch.as_tensor(remapping_array[order], device=pointing.device)
        pointing = torch.as_tensor(inv, device=pointing.device)[torch.searchsorted(ra_sorted, pointing)]
    out = {'tod': cut.tod, 'weights': cut.w, 'keep': keep, 'pointing': pointing, 'az': cut.az, 'el': cut.el,
           'ra': cut.ra, 'dec': cut.dec, 'feedid': cut.feedid, 'obsids': cut.obsid}
    if not device_outputs:
        out = {k: v.cpu().numpy() for k, v in out.items()}
    if remapping_array is None:
        out = _LazyOutputs(out)
        out.lazy('remapping_array', lambda: np.unique(local.cpu().numpy()).astype(int))
    else:
        out['remapping_array'] = remapping_array
    mark('outputs')
    return out


class _LazyOutputs(dict):
    """read_comap_data_bands' result dict with entries computed on first access (a host
    copy the caller may never need).  Every way of reading the dict goes through
    __getitem__: iteration (so dict(r) / {**r} take the keys() + [] path instead of
    copying the raw slots), copy, pop, popitem, setdefault and pickling resolve the
    pending entries first; a pending slot holds a sentinel, never a plausible value."""

    class _Pending:
        def __repr__(self):
            return '<pending lazy value>'

    def lazy(self, key, fn):
        self._lazy = getattr(self, '_lazy', {})
        self._lazy[key] = fn
        dict.__setitem__(self, key, _LazyOutputs._Pending())

    def _resolve(self, key):
        fns = getattr(self, '_lazy', {})
        if key in fns:
            dict.__setitem__(self, key, fns.pop(key)())

    def resolve_all(self):
        for k in list(getattr(self, '_lazy', {})):
            self._resolve(k)
        return self

    def __getitem__(self, key):
        self._resolve(key)
        return dict.__getitem__(self, key)

    def __iter__(self):
        return iter(list(dict.keys(self)))

    def get(self, key, default=None):
        return self[key] if key in self else default

    def items(self):
        return [(k, self[k]) for k in list(self.keys())]

    def values(self):
        return [self[k] for k in list(self.keys())]

    def copy(self):
        return dict(self.resolve_all().items())

    def pop(self, key, *default):
        self._resolve(key)
        return dict.pop(self, key, *default)

    def popitem(self):
        self.resolve_all()
        return dict.popitem(self)

    def setdefault(self, key, default=None):
        self._resolve(key)
        return dict.setdefault(self, key, default)

    def __reduce__(self):
        return (dict, (dict(self.resolve_all().items()),))
