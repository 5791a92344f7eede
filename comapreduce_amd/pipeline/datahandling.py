"""Level-1 / Level-2 data model (host side of the drop-in boundary).

Mirrors the reference's dict-of-datasets classes
(comancpipeline/Analysis/DataHandling.py:40-609): ``HDF5Data``,
``COMAPLevel1``, ``COMAPLevel2`` and ``RepointEdges`` keep the same names,
dataset paths, properties and quirks (scan edges that include the gap,
feature bit decoding, the pre/post-2022 vane temperature).  Datasets may be
NumPy arrays (host) or torch CUDA tensors (device-resident observations, as
bench.py uses); the GPU stages accept both.

HDF5 I/O (the Level-1 / Level-2 wire format) goes through
the native file layer ``pipeline/h5file.py`` -> ``libcomap_h5.so``
(include/comap_h5.h, libhdf5): files are real HDF5, readable by h5py and the
reference.  ``large_datasets`` stay lazy on read (an ``H5Dataset``, as the
reference keeps the h5py Dataset), so a Level-1 cube is staged from the file
straight into pinned buffers on its way to the GPU.  A filename ending in
``.npz`` selects NumPy containers with the same dataset paths instead.
"""
from __future__ import annotations

import itertools
import json
import logging
import os
from dataclasses import dataclass, field
from datetime import datetime, timedelta

import numpy as np
from scipy.interpolate import interp1d

from . import h5file

CALIBRATOR_LIST = ('TauA', 'CasA', 'CygA', 'jupiter', 'sun', 'saturn', 'moon')  # Tools/Coordinates.py:7-15
MJD_EPOCH = datetime(1858, 11, 17)


def mjd_to_datetime(mjd: float) -> datetime:
    return MJD_EPOCH + timedelta(days=float(mjd))


def to_host(x):
    """NumPy view of a dataset (copies torch tensors to the host)."""
    if hasattr(x, 'detach') and hasattr(x, 'cpu'):
        return x.detach().cpu().numpy()
    return np.asarray(x)


@dataclass
class HDF5Data:
    """Dictionary model of an HDF5 file: datasets by path plus per-path attrs."""
    name: str = 'HDF5Data'
    large_datasets: list = field(default_factory=list)
    overwrite: bool = True
    _data: dict = field(default_factory=dict, repr=False)
    _attrs: dict = field(default_factory=dict, repr=False)
    _source: str = ''
    hdf5_file: object = field(default=None, repr=False)   # the open H5File (lazy datasets read from it)

    # No __del__ closing the file: lazy H5Dataset / H5Rows views handed to other
    # containers (sharding.slice_feeds) hold the H5File themselves, and it closes
    # in its own __del__ once the last of them is gone.

    def close(self):
        f, self.hdf5_file = getattr(self, 'hdf5_file', None), None
        if f is not None:
            try:
                f.close()
            except Exception:  # pragma: no cover
                pass

    def __setitem__(self, key, item):
        self._data[key] = item

    def __getitem__(self, key):
        return self._data[key]

    def __contains__(self, key):
        return key in self._data

    def keys(self):
        return self._data.keys()

    def items(self, attr=False):
        return self._attrs.items() if attr else self._data.items()

    def attrs(self, path, attribute_key=None):
        return self._attrs[path] if attribute_key is None else self._attrs[path][attribute_key]

    def set_attrs(self, path, attribute_key, value):
        self._attrs.setdefault(path, {})[attribute_key] = value

    @property
    def filename(self):
        return self._source

    @property
    def groups(self):
        return np.unique([k.split('/')[0] for k in self._data.keys()])

    def create_from_dictionary(self, data: dict, attributes: dict | None = None):
        self._data = dict(data)
        self._attrs = {k: dict(v) for k, v in (attributes or {}).items()}

    # ---------------------------------------------------------------- I/O
    def read_data_file(self, filename: str) -> None:
        """DataHandling.py:101-108, 168-179: every object's attributes, every
        dataset read whole except ``large_datasets`` (kept lazy)."""
        logging.info(f'{self.name}: READING {filename}')
        self._source = filename
        if filename.endswith('.npz'):
            with np.load(filename, allow_pickle=False) as z:
                for k in z.files:
                    if k == '__attrs__':
                        continue
                    self._data[k.replace('|', '/')] = z[k]
                if '__attrs__' in z.files:
                    self._attrs.update(json.loads(str(z['__attrs__'])))
            return
        self.close()
        f = h5file.H5File(filename, 'r')
        self.hdf5_file = f
        for name, kind in f.visit():
            a = f.attrs(name)
            if a:
                self._attrs.setdefault(name, {}).update(a)
            if kind != 'dataset':
                continue
            try:
                self._data[name] = f.dataset(name) if name in self.large_datasets else f.read(name)
            except h5file.H5Error as e:       # a type this layer does not map (e.g. compound)
                logging.warning(f'{self.name}: skipping {name}: {e}')

    def write_data_file(self, filename: str) -> None:
        """DataHandling.py:110-139: append to an existing file (replacing the
        datasets written), skip ``large_datasets``, then the attributes."""
        logging.info(f'{self.name}: WRITING {filename}')
        out = {k: to_host(v) for k, v in self._data.items() if k not in self.large_datasets and v is not None}
        if filename.endswith('.npz'):
            attrs = {k: {a: (v.tolist() if hasattr(v, 'tolist') else v) for a, v in d.items()}
                     for k, d in self._attrs.items()}
            np.savez(filename, __attrs__=json.dumps(attrs, default=str),
                     **{k.replace('/', '|'): v for k, v in out.items()})
            return
        src = self.hdf5_file
        same = src is not None and os.path.abspath(src.filename) == os.path.abspath(filename)
        if same:
            # HDF5 cannot open a file for writing while it is open read-only: close the
            # handle for the write, then re-open it on the same H5File object so every
            # lazy view of it (large_datasets here, H5Rows in shards) reads again
            src.close()
        try:
            self._write_h5(filename, out)
        finally:
            if same:
                src.reopen()
        if self.hdf5_file is None:
            self.hdf5_file = h5file.H5File(filename, 'r')
            self._source = filename

    def _write_h5(self, filename, out):
        with h5file.H5File(filename, 'a' if os.path.exists(filename) else 'w') as h:
            for k, v in out.items():
                h.write(k, v)
            for p, d in self._attrs.items():
                if p not in h:
                    h.require_group(p)
                for a, v in d.items():
                    h.set_attr(p, a, v)


class RepointEdges:
    """Scan finder (reference DataHandling.py:183-245)."""

    @staticmethod
    def get_scan_positions(data, scan_status_code: int = 1):
        if data.source_name in CALIBRATOR_LIST:
            return RepointEdges.get_scan_positions_calibrator(data, scan_status_code)
        return RepointEdges.get_scan_positions_source(data, scan_status_code)

    @staticmethod
    def get_scan_positions_source(data, scan_status_code: int = 1):
        """Pairs (edges[k], edges[k+1]) of the interpolated Lissajous status:
        each scan runs from the previous scan's last sample to its own last
        sample, gap included (DataHandling.py:205-228)."""
        status = to_host(data['hk/antenna0/deTracker/lissajous_status'])
        utc = to_host(data['hk/antenna0/deTracker/utc'])
        mjd = to_host(data['spectrometer/MJD'])
        if np.sum(status) == 0:
            sel = np.where(data.features == 9)[0]
            return np.array([sel[0], sel[-1]]).reshape(1, 2)
        st = interp1d(utc, status, kind='previous', bounds_error=False, fill_value='extrapolate')(mjd)
        on = np.flatnonzero(st == scan_status_code)
        breaks = np.flatnonzero(np.diff(on) > 1)
        edges = on[np.concatenate(([0], breaks, [on.size - 1]))]
        return np.stack([edges[:-1], edges[1:]], axis=1)

    @staticmethod
    def get_scan_positions_calibrator(data, scan_status_code: int = 1):
        idx = np.where(data.on_source)[0]
        return np.array([[int(idx.min())], [int(idx.max())]]).T


def decode_features(f) -> np.ndarray:
    """Feature register -> bit number (int(log2 f), 0 stays 0)."""
    f = np.array(to_host(f), dtype=np.float64)
    nz = f != 0
    f[nz] = np.log(f[nz]) / np.log(2)
    return f.astype(int)


def _source_of(h: HDF5Data, bad_keywords):
    try:
        parts = h.attrs('comap', 'source').split(',')
    except KeyError:
        return ''
    if len(parts) > 1:
        keep = [s for s in parts if s not in bad_keywords]
        return keep[0] if keep else ''
    return parts[0]


@dataclass
class COMAPLevel1(HDF5Data):
    """Level-1 spectrometer file (reference DataHandling.py:248-415)."""
    name: str = 'COMAPLevel1'
    vane_bit_flag: int = 13
    bad_keywords: list = field(default_factory=list)
    OBSID_MINIMUM: int = 7_000
    OBSID_MAXIMUM: int = 1_000_000
    VANE_HOT_TEMP_OFFSET: float = 273.15

    @property
    def obsid(self):
        try:
            return int(self.attrs('comap', 'obsid'))
        except KeyError:
            return -1

    @property
    def comment(self):
        try:
            return self.attrs('comap', 'comment')
        except KeyError:
            return ''

    @property
    def source_name(self):
        return _source_of(self, self.bad_keywords)

    @property
    def features(self):
        if 'spectrometer/features' not in self.keys():
            raise KeyError('LEVEL 1 FILE CONTAINS NO: spectrometer/features')
        return decode_features(self['spectrometer/features'])

    @property
    def on_source(self):
        f = self.features
        return (f != 13) & (f != 0) & (f != 16)

    @property
    def vane_flag(self):
        return self.features == self.vane_bit_flag

    @property
    def vane_temperature(self):
        date = mjd_to_datetime(to_host(self['spectrometer/MJD'])[0])
        if date < datetime(2022, 2, 1):
            return np.nanmean(to_host(self['hk/antenna0/vane/Tvane'])) / 100.0 + self.VANE_HOT_TEMP_OFFSET
        tshroud = np.nanmean(to_host(self['hk/antenna0/vane/Tshroud'])) / 100.0 + self.VANE_HOT_TEMP_OFFSET
        return 0.2702 * tshroud + 213

    @property
    def tod_shape(self):
        return tuple(self['spectrometer/tod'].shape)

    @property
    def frequency(self):
        return self['spectrometer/frequency']

    @property
    def scan_edges(self):
        cached = getattr(self, '_scan_edges_cache', None)
        if cached is None:
            cached = RepointEdges.get_scan_positions(self)
            self._scan_edges_cache = cached
        return cached

    ra = property(lambda s: s['spectrometer/pixel_pointing/pixel_ra'])
    dec = property(lambda s: s['spectrometer/pixel_pointing/pixel_dec'])
    az = property(lambda s: s['spectrometer/pixel_pointing/pixel_az'])
    el = property(lambda s: s['spectrometer/pixel_pointing/pixel_el'])

    @property
    def airmass(self):
        el = to_host(self.el)
        return 1.0 / np.sin(el * np.pi / 180.0)

    def tod_loop(self, feeds=True, bands=True, channels=True):
        n_feeds, n_bands, n_channels, _ = self.tod_shape
        its = []
        if feeds:
            its.append(np.vstack([np.arange(n_feeds, dtype=int), to_host(self['spectrometer/feeds'])]).T)
        if bands:
            its.append(np.arange(n_bands, dtype=int))
        if channels:
            its.append(np.arange(n_bands, dtype=int))   # sic: the reference iterates bands here
        return itertools.product(*its)


class COMAPLevel2(HDF5Data):
    """Level-2 output file (reference DataHandling.py:417-609)."""

    def __init__(self, filename: str = 'pipeline_output.hdf5', **kw):
        super().__init__(name=kw.pop('name', 'COMAPLevel2'), **{k: v for k, v in kw.items()
                                                                 if k in ('large_datasets', 'overwrite')})
        self.filename_ = filename
        self.vane_bit_flag = 13
        self.bad_keywords = kw.get('bad_keywords', [])
        for cand in (filename, filename + '.npz'):
            if os.path.exists(cand):
                self.read_data_file(cand)
                break

    def contains(self, pipeline_function) -> bool:
        return all(g.split('/')[0] in self.groups for g in pipeline_function.groups)

    def update(self, pipeline_function) -> None:
        data, attrs = pipeline_function.save_data
        for k, v in data.items():
            if v is not None:
                self[k] = v
        for k, v in attrs.items():
            for a, val in v.items():
                self.set_attrs(k, a, val)

    @property
    def source_name(self):
        return _source_of(self, self.bad_keywords)

    @property
    def obsid(self):
        try:
            return int(self.attrs('comap', 'obsid'))
        except KeyError:
            return -1

    @property
    def features(self):
        return decode_features(self['spectrometer/features'])

    @property
    def vane_flag(self):
        return self.features == self.vane_bit_flag

    @property
    def on_source(self):
        f = self.features
        return (f != 13) & (f != 0)

    @property
    def scan_edges(self):
        if 'averaged_tod/scan_edges' in self.keys():
            return self['averaged_tod/scan_edges']
        return RepointEdges.get_scan_positions(self)

    @property
    def tod_shape(self):
        return tuple(self['averaged_tod/tod'].shape)

    @property
    def nbands(self):
        return self.tod_shape[1]

    feeds = property(lambda s: s['spectrometer/feeds'])
    tod = property(lambda s: s['averaged_tod/tod'], lambda s, v: s.__setitem__('averaged_tod/tod', v))
    mjd = property(lambda s: s['spectrometer/MJD'], lambda s, v: s.__setitem__('spectrometer/MJD', v))
    ra = property(lambda s: s['spectrometer/pixel_pointing/pixel_ra'])
    dec = property(lambda s: s['spectrometer/pixel_pointing/pixel_dec'])
    az = property(lambda s: s['spectrometer/pixel_pointing/pixel_az'])
    el = property(lambda s: s['spectrometer/pixel_pointing/pixel_el'])
    system_temperature = property(lambda s: s['vane/system_temperature'],
                                  lambda s, v: s.__setitem__('vane/system_temperature', v))
    system_gain = property(lambda s: s['vane/system_gain'], lambda s, v: s.__setitem__('vane/system_gain', v))

    @property
    def airmass(self):
        return 1.0 / np.sin(to_host(self.el) * np.pi / 180.0)

    def tod_auto_rms(self, ifeed: int, iband: int):
        tod = to_host(self['averaged_tod/tod'])[ifeed, iband]
        t = tod[tod != 0]
        N = t.size // 2 * 2
        return np.nanstd(t[:N:2] - t[1:N:2]) / np.sqrt(2)

    def tod_loop(self, feeds=True, bands=True):
        n_feeds, n_bands, _ = self.tod_shape
        its = []
        if feeds:
            its.append(np.vstack([np.arange(n_feeds, dtype=int), to_host(self['spectrometer/feeds'])]).T)
        if bands:
            its.append(np.arange(n_bands, dtype=int))
        return itertools.product(*its)


def level1_from_dict(gen: dict, level=COMAPLevel1) -> COMAPLevel1:
    """Builds a COMAPLevel1 from {'data':..., 'attrs':...} (synthetic generator output)."""
    d = level(overwrite=False, large_datasets=['spectrometer/tod'])
    for k, v in gen['data'].items():
        d[k] = v
    for p, a in gen.get('attrs', {}).items():
        for k, v in a.items():
            d.set_attrs(p, k, v)
    return d
