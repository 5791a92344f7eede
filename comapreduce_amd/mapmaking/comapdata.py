"""Destriper data prep: Level-2 files -> flat (tod, weights, pointing, ...) vectors.

Mirror of reference comancpipeline/MapMaking/COMAPData.py (same function
names, arguments and outputs).  The per-sample host work is vectorised over
feeds and scans; the one expensive step -- the reflect-padded 400-sample
running median subtracted from every (feed, scan) series (get_tod,
COMAPData.py:353-360) -- is collected for ALL files of the rank and run in a
single ``comap_medfilt_batch_f64`` device call (exact selection, bit-identical
to medianFilter.cpp).  There is no CPU fallback for that call.

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


class _FilePrep:
    """get_tod (COMAPData.py:247-380) split in two: ``collect`` builds the
    per-feed arrays and queues median-filter series; ``finish`` subtracts the
    filtered baselines once the batched device call has run."""

    def __init__(self, f, datasize, offset_length, selected_feeds, use_gain_filter, iband, calibration,
                 calibrator, queue):
        source = f.attrs('comap')['source'].split(',')[0]
        self.calib_source = source in CALIBRATORS
        dset = f['averaged_tod/tod'] if (use_gain_filter and not self.calib_source) else f['averaged_tod/tod_original']
        bad_feeds = f.attrs('comap')['bad_observation']
        spike = f['spikes/spike_mask'] if 'spikes/spike_mask' in f else None
        if spike is not None and np.ndim(spike) == 1:
            spike = None
        file_feeds = np.asarray(f['spectrometer/feeds'])
        if calibration:
            cal = np.zeros((20, 4))
            for b in range(4):
                cal[:, b] = f.attrs('comap')[f'{calibrator}_calibration_factor_band{b}']
        else:
            cal = np.ones(dset.shape[:2])
        fi, oi = GetFeeds(file_feeds, selected_feeds)
        shape = (len(oi), datasize)
        self.tod, self.weights, self.az, self.el, self.ra, self.dec = (np.zeros(shape) for _ in range(6))
        self.feedid = np.zeros(shape)
        self.edges = get_scan_edges(f)
        self.lens = scan_lengths(self.edges, offset_length)
        self.pending = []                       # (tod_file, start, N, ~bad index, queue slot | None, value)
        if len(self.edges) == 0:
            return
        mjd0 = f['spectrometer/MJD'][0]
        for ff, of in zip(fi, oi):
            if feed_is_bad(bad_feeds[file_feeds[ff]]):
                continue
            tod_file = dset[ff, iband, :] / cal[ff, iband]
            w_file = np.ones(tod_file.size) / auto_rms(tod_file) ** 2
            az_f = np.asarray(f['spectrometer/pixel_pointing/pixel_az'][ff, :])
            el_f = np.asarray(f['spectrometer/pixel_pointing/pixel_el'][ff, :])
            ra_f, dec_f = astro.sun_distance_deg(f['spectrometer/pixel_pointing/pixel_ra'][ff, :],
                                                 f['spectrometer/pixel_pointing/pixel_dec'][ff, :], mjd0)
            self.feedid[of] = file_feeds[ff]
            if spike is not None:
                w_file[spike[ff, iband, :]] = 0
            w_file[ra_f < 10] = 0
            good = np.isfinite(az_f)
            az10, az90 = np.percentile(az_f[good], 10), np.percentile(az_f[good], 90)
            el10, el90 = np.percentile(el_f[good], 10), np.percentile(el_f[good], 90)
            w_file[(az_f < az10) | (az_f > az90)] = 0
            w_file[(el_f < el10) | (el_f > el90)] = 0
            last = 0
            for (start, _), N in zip(self.edges, self.lens):
                Nten = int(N * 0.1)
                w_file[start:start + Nten] = 0
                w_file[start + N - Nten:start + N] = 0
                if not self.calib_source:
                    seg = tod_file[start:start + N]
                    # the reference passes non-finite samples to medianFilter.cpp, whose
                    # two-heap order is undefined for NaN; they end with tod = 0 and
                    # weight 0 (COMAPData.py:550-552), so here they are left out of the
                    # median input (parity for series holding NaN is unpinned)
                    keep = np.nonzero((seg != 0) & np.isfinite(seg))[0]
                    vals = seg[keep]
                    if vals.size > 2 * MEDFILT_STEP:
                        slot = len(queue)
                        queue.append(vals)
                        self.pending.append((of, last, keep, slot, None))
                    else:
                        self.pending.append((of, last, keep, None, np.ones(vals.size) * np.nanmedian(vals)))
                self.tod[of, last:last + N] = tod_file[start:start + N]
                self.weights[of, last:last + N] = w_file[start:start + N]
                self.az[of, last:last + N] = az_f[start:start + N]
                self.el[of, last:last + N] = el_f[start:start + N]
                self.ra[of, last:last + N] = ra_f[start:start + N]
                self.dec[of, last:last + N] = dec_f[start:start + N]
                last += N

    def finish(self, filtered):
        for of, last, keep, slot, val in self.pending:
            base = filtered[slot] if slot is not None else val
            row = self.tod[of]
            row[last + keep] -= base
        return (self.tod.ravel(), self.weights.ravel(), self.az.ravel(), self.el.ravel(), self.ra.ravel(),
                self.dec.ravel(), self.feedid.ravel().astype(int))


def read_comap_data(filelist, map_info, feed_weights=None, iband=0, use_gain_filter=True, offset_length=50,
                    feeds=[i + 1 for i in range(19)], calibration=False, calibrator='TauA', healpix=False,
                    store=None, device=None):
    """COMAPData.read_comap_data (COMAPData.py:471-577): same arguments and
    return tuple ``(tod, weights, pointing, remapping_array, az, el, ra, dec,
    feedid, obsids)``.  ``store`` (tests) maps filename -> (datasets, attrs);
    ``device``: the rank's GPU for the batched median (default: torch's
    current device)."""
    (tod,), (weights,), pointing, az, el, ra, dec, feedid, obsids = _read_uncut(
        filelist, map_info, (iband,), use_gain_filter, offset_length, feeds, calibration, calibrator, store, device,
        healpix)
    mask = ~np.isfinite(tod)
    tod[mask] = 0
    weights[mask] = 0
    keep = np.repeat((weights != 0).reshape(-1, offset_length).any(axis=1), offset_length)
    tod, weights, pointing = tod[keep], weights[keep], pointing[keep]
    az, el, ra, dec, feedid, obsids = az[keep], el[keep], ra[keep], dec[keep], feedid[keep], obsids[keep]
    weights[~np.isfinite(weights)] = 0
    remapping_array = find_unique_values(np.unique(pointing))
    if healpix:      # COMAPData.py:572-573: pixel ids -> positions in the union over ranks
        from .healpix import index_replace
        pointing = index_replace(remapping_array, pointing)
    return tod, weights, pointing, remapping_array.astype(int), az, el, ra, dec, feedid, obsids


def _read_uncut(filelist, map_info, bands, use_gain_filter, offset_length, feeds, calibration, calibrator, store,
                device, healpix=False):
    """Per-band tod / weights (lists) and the band-independent vectors of
    read_comap_data before its NaN and empty-offset cuts.  Every band's
    400-sample high-pass series of every file go through ONE batched device
    median call."""
    from ..tools.medfilt import medfilt_batch
    open_file = _opener(store)
    Nfeeds = len(feeds)
    files = [open_file(fn) for fn in filelist]
    sizes = [countDataSize(f, Nfeeds, offset_length) for f in files]
    queue, preps, pix = [], [], []
    for fn, f, info in zip(filelist, files, sizes):
        ds = int(info['datasize'])
        pix.append((read_pixels_healpix if healpix else read_pixels)(f, ds, offset_length, feeds, map_info))
        preps.append([_FilePrep(f, ds, offset_length, feeds, use_gain_filter, b, calibration, calibrator, queue)
                      for b in bands])
    filtered = medfilt_batch(queue, MEDFILT_STEP, reflect=True, device=device)
    parts = [[p.finish(filtered) for p in per_band] for per_band in preps]
    N = sum(i['N'] for i in sizes)
    tods = [np.zeros(N) for _ in bands]
    wts = [np.zeros(N) for _ in bands]
    az, el, ra, dec = (np.zeros(N) for _ in range(4))
    pointing = np.zeros(N, dtype=int)
    feedid = np.zeros(N, dtype=int)
    obsids = np.zeros(N, dtype=int)
    last = 0
    for fn, outs, p in zip(filelist, parts, pix):
        n = outs[0][0].size
        for k, out in enumerate(outs):
            tods[k][last:last + n] = out[0]
            wts[k][last:last + n] = out[1]
        for arr, v in zip((az, el, ra, dec, feedid), outs[0][2:]):
            arr[last:last + n] = v
        pointing[last:last + n] = p.ravel()
        obsids[last:last + n] = int(os.path.basename(fn).split('-')[1])
        last += n
    return tods, wts, pointing, az, el, ra, dec, feedid, obsids


def read_comap_data_bands(filelist, map_info, bands=(0, 1, 2, 3), use_gain_filter=True, offset_length=50,
                          feeds=[i + 1 for i in range(19)], calibration=False, calibrator='TauA', healpix=False,
                          store=None, device=None):
    """read_comap_data for several bands at once, for the batched destriper
    (run_destriper.py:146-189 calls read_comap_data once per band on the same
    files; only tod and weights depend on the band).

    Each band gets the reference's NaN cut (tod and weight 0).  The reference
    then drops the offsets whose weights are all zero -- per band, so the
    bands' sample sets differ; here the samples of every offset that ANY band
    keeps are returned, with keep[b, o] saying whether band b's own
    read_comap_data would have kept offset o (its weights there are all 0 when
    not).  Band b's kept samples, in order, are exactly what
    read_comap_data(iband=b) returns.

    Returns dict: tod, weights [nb, N]; keep uint8 [nb, N/L]; pointing, az, el,
    ra, dec, feedid, obsids [N]; remapping_array (unique pixels of the union)."""
    tods, wts, pointing, az, el, ra, dec, feedid, obsids = _read_uncut(
        filelist, map_info, tuple(bands), use_gain_filter, offset_length, feeds, calibration, calibrator, store,
        device, healpix)
    keeps = []
    for t, w in zip(tods, wts):
        bad = ~np.isfinite(t)
        t[bad] = 0
        w[bad] = 0
        keeps.append((w != 0).reshape(-1, offset_length).any(axis=1))
    keep = np.stack(keeps) if keeps else np.zeros((0, pointing.size // offset_length), dtype=bool)
    union = keep.any(axis=0)
    sel = np.repeat(union, offset_length)
    tod = np.stack([t[sel] for t in tods])
    weights = np.stack([w[sel] for w in wts])
    weights[~np.isfinite(weights)] = 0
    pointing = pointing[sel]
    out = {'tod': tod, 'weights': weights, 'keep': keep[:, union].astype(np.uint8), 'pointing': pointing,
           'az': az[sel], 'el': el[sel], 'ra': ra[sel], 'dec': dec[sel], 'feedid': feedid[sel],
           'obsids': obsids[sel]}
    out['remapping_array'] = find_unique_values(np.unique(pointing)).astype(int)
    if healpix:
        from .healpix import index_replace
        out['pointing'] = index_replace(out['remapping_array'], pointing)
    return out
