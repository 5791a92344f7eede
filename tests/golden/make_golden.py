#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE (COMAPreduce v0.9.1) here.

This script is test infrastructure and runs only in the build container, where
/root/reference exists.  It never travels to the GPU box; only its small
outputs (tests/golden/*.npz, *.json) are committed.

What it does
------------
1. Copies /root/reference/comancpipeline to a scratch dir (/tmp) -- the
   reference source is never copied into this repository.
2. Compiles the reference's own Cython/C++ helpers there, unmodified:
   Tools/binFuncs.pyx and Tools/median_filter/medfilt.pyx (+ medianFilter.cpp,
   Mediator.h) with cythonize + g++.
3. Imports the reference Analysis/MapMaking modules with sys.modules stand-ins
   for imports that are absent from this image and are NOT on the numeric path
   being pinned:
     mpi4py  -> single-rank COMM_WORLD (rank 0, size 1; Allreduce/Reduce copy,
                Gather/Bcast identity) -- the reference's own 1-rank behaviour;
     h5py    -> only the File/Dataset names (no file I/O is performed);
     astropy.time.Time -> MJD->datetime (used only for the vane-temperature
                date branch, DataHandling.py:316-326);
     healpy, astropy.{wcs,io,coordinates}, astroplan, toml, Tools.pysla ->
                empty modules (imported at module level, unused on this path).
   The stages are driven directly on in-memory COMAPLevel1/COMAPLevel2 objects
   (Runner.run_tod needs h5py); spectrometer/tod is wrapped so every slice is a
   fresh copy, as an h5py Dataset would return (SURVEY.md §8a parity notes).
4. Writes:
   golden_l1_c1.npz      MeasureSystemTemperature -> AtmosphereRemoval ->
                         Level1AveragingGainCorrection on the C1 synthetic
                         observation (1 feed x 4 x 1024 x 30,000)
   golden_medfilt.npz    medfilt.medfilt known-answer tests
   golden_binvalues.npz  binFuncs.binValues known-answer tests
   golden_destriper.npz  Destriper.destriper_iteration on a small problem
   golden_binning.npz    Level1Averaging.average_tod on the C1 observation (strided)
   golden_noise.npz      Level2FitPowerSpectrum + NoiseStatistics (variants.noise_level2)
   golden_meta.json      input SHA-256s, reference timings, provenance

Usage:  python tests/golden/make_golden.py [--skip-l1 | --only-variants | --only-comapdata | --only-binning | --only-noise]
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import time
import types
from datetime import datetime, timedelta

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
SCRATCH = '/tmp/comap_ref_golden'

sys.path.insert(0, REPO)
from comapreduce_amd import synthetic  # noqa: E402

MEDFILT_CASES = [  # (seed, n, w)
    (11, 40_000, 6000), (12, 20_000, 400), (13, 5_000, 100), (14, 9_000, 401),
    (15, 3_001, 7), (16, 2_000, 1), (17, 1_000, 2), (18, 45_000, 6000),
]


def build_reference_helpers():
    if os.path.isdir(SCRATCH):
        shutil.rmtree(SCRATCH)
    shutil.copytree(os.path.join(REF, 'comancpipeline'), os.path.join(SCRATCH, 'comancpipeline'),
                    ignore=shutil.ignore_patterns('__pycache__', '*.so'))
    setup = """
from setuptools import setup, Extension
from Cython.Build import cythonize
import numpy
ext = [Extension('comancpipeline.Tools.binFuncs', ['comancpipeline/Tools/binFuncs.pyx'],
                 include_dirs=[numpy.get_include()]),
       Extension('comancpipeline.Tools.median_filter.medfilt',
                 ['comancpipeline/Tools/median_filter/medfilt.pyx'],
                 include_dirs=[numpy.get_include(), 'comancpipeline/Tools/median_filter'],
                 language='c++', extra_compile_args=['-fopenmp'], extra_link_args=['-fopenmp'])]
setup(ext_modules=cythonize(ext, language_level=3, quiet=True))
"""
    with open(os.path.join(SCRATCH, 'setup_golden.py'), 'w') as f:
        f.write(setup)
    subprocess.run([sys.executable, 'setup_golden.py', 'build_ext', '--inplace', '-q'],
                   cwd=SCRATCH, check=True, stdout=subprocess.DEVNULL)


class _Comm:
    def Get_rank(self): return 0
    def Get_size(self): return 1
    def Barrier(self): pass
    def Allreduce(self, a, b, op=None):
        src = a[0] if isinstance(a, (list, tuple)) else a
        dst = b[0] if isinstance(b, (list, tuple)) else b
        np.copyto(dst, np.asarray(src).reshape(np.shape(dst)))
    def Reduce(self, a, b, op=None, root=0): np.copyto(b, a)
    def Gather(self, a, b, root=0):
        if b is not None:
            b[...] = np.asarray(a).reshape(np.shape(b))
    def Bcast(self, a, root=0): pass
    def allgather(self, x): return [x]
    def allreduce(self, x, op=None): return x


def install_stubs():
    mpi = types.ModuleType('mpi4py')
    MPI = types.ModuleType('mpi4py.MPI')
    MPI.COMM_WORLD = _Comm()
    MPI.SUM, MPI.MAX, MPI.DOUBLE = 'sum', 'max', 'double'
    mpi.MPI = MPI
    sys.modules['mpi4py'] = mpi
    sys.modules['mpi4py.MPI'] = MPI
    h5 = types.ModuleType('h5py')
    h5.File = type('File', (), {})
    h5.Dataset = type('Dataset', (), {})
    sys.modules['h5py'] = h5

    class Time:
        def __init__(self, v, format='mjd'):
            self.datetime = datetime(1858, 11, 17) + timedelta(days=float(np.asarray(v).ravel()[0]))

    class _Dummy:
        def __init__(self, *a, **k): pass
        def __call__(self, *a, **k): return _Dummy()
        def __getattr__(self, name): return _Dummy()

    class StubModule(types.ModuleType):
        __path__ = []
        def __getattr__(self, name):
            if name.startswith('__'):
                raise AttributeError(name)
            return _Dummy

    import importlib.abc
    import importlib.machinery

    class StubFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
        prefixes = ('astropy', 'healpy', 'astroplan', 'toml', 'emcee', 'comancpipeline.Tools.pysla')
        def find_spec(self, fullname, path, target=None):
            if any(fullname == p or fullname.startswith(p + '.') for p in self.prefixes):
                return importlib.machinery.ModuleSpec(fullname, self)
            return None
        def create_module(self, spec):
            return StubModule(spec.name)
        def exec_module(self, module):
            if module.__name__ == 'astropy.time':
                module.Time = Time
    sys.meta_path.insert(0, StubFinder())
    sys.path.insert(0, SCRATCH)
    sys.path.insert(0, os.path.join(SCRATCH, 'comancpipeline', 'MapMaking'))


class CopyOnSlice:
    """Mimics an h5py Dataset: every slice is a fresh ndarray copy."""

    def __init__(self, arr):
        self._a = arr
        self.shape = arr.shape
        self.dtype = arr.dtype

    def __getitem__(self, idx):
        return np.array(self._a[idx])


def run_l1(out, meta, figdir):
    from comancpipeline.Analysis.DataHandling import COMAPLevel1, COMAPLevel2
    from comancpipeline.Analysis.VaneCalibration import MeasureSystemTemperature
    from comancpipeline.Analysis.Level1Averaging import AtmosphereRemoval, Level1AveragingGainCorrection

    cfg = synthetic.SyntheticConfig(n_feeds=1, n_samples=30_000, obs_id=1)
    gen = synthetic.generate_level1(cfg)
    meta['l1_c1_config'] = dict(n_feeds=1, n_samples=30_000, obs_id=1)
    meta['l1_c1_sha256'] = {k: synthetic.sha256(v) for k, v in gen['data'].items()}

    data = COMAPLevel1(overwrite=False, large_datasets=['spectrometer/tod'])
    for k, v in gen['data'].items():
        data[k] = CopyOnSlice(v) if k == 'spectrometer/tod' else v
    for k, v in gen['attrs']['comap'].items():
        data.set_attrs('comap', k, v)
    level2 = COMAPLevel2(filename=os.path.join(figdir, 'does_not_exist.hd5'))

    timings = {}
    for cls in (MeasureSystemTemperature, AtmosphereRemoval, Level1AveragingGainCorrection):
        stage = cls(level2=level2, figure_directory=figdir)
        t0 = time.perf_counter()
        ok = stage(data, level2)
        timings[cls.__name__] = time.perf_counter() - t0
        assert ok, cls.__name__
        level2.update(stage)
    meta['reference_timings_s_c1'] = timings
    meta['reference_samples_channels_c1'] = int(1 * 4 * 1024 * 30_000)
    for k in ('vane/system_temperature', 'vane/system_gain', 'atmosphere/fit_values',
              'averaged_tod/tod', 'averaged_tod/tod_original', 'averaged_tod/weights',
              'averaged_tod/scan_edges', 'averaged_tod/frequency_power_spectra',
              'averaged_tod/frequency_power_spectra_fits'):
        out[k.replace('/', '__')] = np.asarray(level2[k])


def run_l1_variant(name, figdir):
    """Edge-case observations (tests/golden/variants.py) through the same three stages."""
    from comancpipeline.Analysis.DataHandling import COMAPLevel1, COMAPLevel2
    from comancpipeline.Analysis.VaneCalibration import MeasureSystemTemperature
    from comancpipeline.Analysis.Level1Averaging import AtmosphereRemoval, Level1AveragingGainCorrection
    sys.path.insert(0, HERE)
    import variants
    gen = variants.make(name)
    data = COMAPLevel1(overwrite=False, large_datasets=['spectrometer/tod'])
    for k, v in gen['data'].items():
        data[k] = CopyOnSlice(v) if k == 'spectrometer/tod' else v
    for k, v in gen['attrs']['comap'].items():
        data.set_attrs('comap', k, v)
    level2 = COMAPLevel2(filename=os.path.join(figdir, 'does_not_exist.hd5'))
    for cls in (MeasureSystemTemperature, AtmosphereRemoval, Level1AveragingGainCorrection):
        stage = cls(level2=level2, figure_directory=figdir)
        assert stage(data, level2), cls.__name__
        level2.update(stage)
    out = {}
    for k in ('vane/system_temperature', 'vane/system_gain', 'atmosphere/fit_values',
              'averaged_tod/tod', 'averaged_tod/tod_original', 'averaged_tod/weights',
              'averaged_tod/scan_edges'):
        v = np.asarray(level2[k])
        if name == 'f3' and k in ('averaged_tod/tod', 'averaged_tod/tod_original', 'averaged_tod/weights'):
            v = v[..., ::variants.F3_STRIDE]
        out[k.replace('/', '__')] = v
    np.savez_compressed(os.path.join(HERE, f'golden_l1_{name}.npz'), **out)
    return {k: synthetic.sha256(v) for k, v in gen['data'].items()}


def run_spikes():
    """Statistics.Spikes (Statistics.py:31-105) on a Level-2 TOD with injected spikes."""
    from comancpipeline.Analysis.DataHandling import COMAPLevel2
    from comancpipeline.Analysis.Statistics import Spikes
    sys.path.insert(0, HERE)
    import variants
    tod, edges = variants.spikes_level2(HERE)
    l2 = COMAPLevel2(filename='/nonexistent/spikes.hd5')
    l2['averaged_tod/tod'] = tod
    l2['averaged_tod/scan_edges'] = edges
    l2['spectrometer/feeds'] = np.array([1])
    l2.set_attrs('comap', 'source', 'Field00')
    st = Spikes(level2=l2)
    assert st(l2, l2)
    np.savez_compressed(os.path.join(HERE, 'golden_spikes.npz'), spike_mask=st.data['spikes/spike_mask'])


def run_noise():
    """Level2FitPowerSpectrum (Level2Data.py:224-329) and NoiseStatistics
    (Statistics.py:107-224) on the noise-QA Level-2 input (variants.noise_level2)."""
    from comancpipeline.Analysis.DataHandling import COMAPLevel2
    from comancpipeline.Analysis.Level2Data import Level2FitPowerSpectrum
    from comancpipeline.Analysis.Statistics import NoiseStatistics
    sys.path.insert(0, HERE)
    import variants
    tod, edges, mask, feeds = variants.noise_level2(HERE)
    figdir = os.path.join(SCRATCH, 'figures_noise')
    os.makedirs(figdir, exist_ok=True)
    out = {'tod': tod, 'scan_edges': edges, 'spike_mask': mask, 'feeds': feeds}
    timings = {}
    l2 = COMAPLevel2(filename='/nonexistent/noise.hd5')
    l2['averaged_tod/tod'] = tod
    l2['averaged_tod/scan_edges'] = edges
    l2['spectrometer/feeds'] = feeds
    l2.set_attrs('comap', 'source', 'Field00')
    l2.set_attrs('comap', 'obsid', 1)
    st = Level2FitPowerSpectrum(level2=l2, figure_directory=figdir)
    t0 = time.perf_counter()
    assert st(l2, l2)
    timings['Level2FitPowerSpectrum'] = time.perf_counter() - t0
    out['fnoise_fit_parameters'] = st.data['fnoise_fits/fnoise_fit_parameters']
    out['fnoise_auto_rms'] = st.data['fnoise_fits/auto_rms']
    for with_mask in (False, True):
        l2n = COMAPLevel2(filename='/nonexistent/noise.hd5')
        l2n['averaged_tod/tod'] = tod
        l2n['averaged_tod/scan_edges'] = edges
        l2n['spectrometer/feeds'] = feeds
        if with_mask:
            l2n['spikes/spike_mask'] = mask
        l2n.set_attrs('comap', 'source', 'Field00')
        ns = NoiseStatistics(level2=l2n)
        t0 = time.perf_counter()
        assert ns(l2n, l2n)
        timings[f'NoiseStatistics_mask{int(with_mask)}'] = time.perf_counter() - t0
        out[f'fnoise_mask{int(with_mask)}'] = ns.data['noise_statistics/fnoise']
    np.savez_compressed(os.path.join(HERE, 'golden_noise.npz'), **out)
    return timings


class _FakeH5:
    """h5py.File stand-in over an in-memory (datasets, attrs) pair."""

    def __init__(self, entry):
        self._d, self._a = entry

    def __getitem__(self, k):
        if k in self._a and k not in self._d:
            return types.SimpleNamespace(attrs=self._a[k])
        return CopyOnSlice(np.asarray(self._d[k]))

    def __contains__(self, k):
        return k in self._d

    def close(self):
        pass


def run_comapdata():
    """MapMaking/COMAPData.read_comap_data on three synthetic Level-2 files.

    Leaves absent from this image are replaced by the repo's restatements
    (astropy WCS -> comapreduce_amd.mapmaking.wcs.CelestialWCS; healpy
    Rotator -> mapmaking.astro.Rotator; astropy get_sun -> astro.sun_radec);
    everything else (file/feed/scan loops, auto_rms, cuts, 400-sample median
    via the compiled medianFilter.cpp, flattening, empty-offset cut) is the
    reference's own code."""
    import COMAPData
    from comapreduce_amd.mapmaking import astro
    from comapreduce_amd.mapmaking.wcs import CelestialWCS
    sys.path.insert(0, HERE)
    import comapdata_case as cc
    store, names = cc.store()
    COMAPData.h5py = types.SimpleNamespace(File=lambda fn, mode='r': _FakeH5(store[fn]))
    COMAPData.hp = types.SimpleNamespace(rotator=types.SimpleNamespace(Rotator=astro.Rotator))
    COMAPData.Time = lambda v, format='mjd': types.SimpleNamespace(mjd=float(v))

    def get_sun(t):
        ra, dec = astro.sun_radec(t.mjd)
        return types.SimpleNamespace(ra=types.SimpleNamespace(deg=ra), dec=types.SimpleNamespace(deg=dec))
    COMAPData.get_sun = get_sun
    out = {}
    for name, case in cc.CASES.items():
        m = case['map']
        map_info = {'wcs': CelestialWCS(m['crval'], m['cdelt'], m['crpix'], m['ctype']),
                    'nxpix': m['nxpix'], 'nypix': m['nypix']}
        res = COMAPData.read_comap_data(np.array(names), map_info, feeds=cc.FEEDS, **case['kw'])
        for k, v in zip(cc.OUTPUTS, res):
            out[f'{name}__{k}'] = np.asarray(v)[::cc.STRIDE] if k in cc.STRIDED else np.asarray(v)
    np.savez_compressed(os.path.join(HERE, 'golden_comapdata.npz'), **out)
    return {n: {k: synthetic.sha256(np.asarray(v)) for k, v in store[n][0].items()} for n in names}


def run_parser():
    """Tools/ParserClass.Parser on tests/golden/params_case.ini (our own fixture)."""
    from comancpipeline.Tools import ParserClass
    from comancpipeline.Tools import Coordinates
    p = ParserClass.Parser(os.path.join(HERE, 'params_case.ini'))
    return {'parsed': p.infodict,
            'sex2deg': [Coordinates.sex2deg('11:20:00', hours=True), Coordinates.sex2deg('+52:00:00'),
                        Coordinates.sex2deg('-00:30:36'), Coordinates.sex2deg('05:32:00.3', hours=True)]}


BINNING_STRIDE = 7    # golden_binning.npz keeps every 7th sample of the C1 outputs


def run_binning():
    """Level1Averaging.average_tod (Level1Averaging.py:292-321) on the C1 observation,
    with the vane solution of the reference's own MeasureSystemTemperature.  The
    stage's __call__(data) is unreachable from Runner (:275), so average_tod is
    called directly, as a user would."""
    from comancpipeline.Analysis.DataHandling import COMAPLevel1, COMAPLevel2
    from comancpipeline.Analysis.VaneCalibration import MeasureSystemTemperature
    from comancpipeline.Analysis.Level1Averaging import Level1Averaging
    figdir = os.path.join(SCRATCH, 'figures')
    os.makedirs(figdir, exist_ok=True)
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(n_feeds=1, n_samples=30_000, obs_id=1))
    data = COMAPLevel1(overwrite=False, large_datasets=['spectrometer/tod'])
    for k, v in gen['data'].items():
        data[k] = CopyOnSlice(v) if k == 'spectrometer/tod' else v
    for k, v in gen['attrs']['comap'].items():
        data.set_attrs('comap', k, v)
    level2 = COMAPLevel2(filename=os.path.join(figdir, 'does_not_exist.hd5'))
    vane = MeasureSystemTemperature(level2=level2, figure_directory=figdir)
    assert vane(data, level2)
    level2.update(vane)
    st = Level1Averaging(level2=level2)
    st.average_tod(data)
    np.savez_compressed(os.path.join(HERE, 'golden_binning.npz'), stride=BINNING_STRIDE,
                        tod=st.tod[..., ::BINNING_STRIDE], tod_stddev=st.tod_stddev[..., ::BINNING_STRIDE])


def run_medfilt(out):
    from comancpipeline.Tools.median_filter import medfilt
    for seed, n, w in MEDFILT_CASES:
        x = np.random.default_rng(seed).standard_normal(n)
        y = np.array(medfilt.medfilt(x.copy(), np.int32(w)))
        out[f'medfilt_{seed}_{n}_{w}'] = y


def run_binvalues(out):
    from comancpipeline.Tools import binFuncs
    rng = np.random.default_rng(21)
    npix = 1000
    pix = rng.integers(-50, npix + 50, 50_000).astype(np.int64)
    w = rng.standard_normal(50_000)
    mask = (rng.random(50_000) > 0.3).astype(np.int64)
    img = np.zeros(npix); binFuncs.binValues(img, pix, weights=w)
    out['binvalues_weighted'] = img
    img = np.zeros(npix); binFuncs.binValues(img, pix)
    out['binvalues_hits'] = img
    img = np.zeros(npix); binFuncs.binValues(img, pix, weights=w, mask=mask)
    out['binvalues_masked'] = img


def run_destriper(out, meta):
    import Destriper
    L = 50
    pointing, tod, weights = synthetic.destriper_inputs()
    npix = 60 * 60
    pixel_edges = np.arange(npix)
    z = np.zeros(tod.size)
    feedid = np.repeat([1, 2], tod.size // 2)
    obsids = np.ones(tod.size, dtype=int)
    t0 = time.perf_counter()
    maps, result, _ = Destriper.destriper_iteration(pointing, z, tod, weights, L, pixel_edges,
                                                    feedid, obsids, threshold=1e-6, niter=100)
    meta['reference_destriper_s'] = time.perf_counter() - t0
    out['destriper_offsets'] = result
    for k in ('map', 'naive', 'weight', 'hits'):
        out[f'destriper_{k}'] = maps[k]
    # fixed-iteration variant (no early exit) for iterate-level parity
    maps5, result5, _ = Destriper.destriper_iteration(pointing, z, tod, weights, L, pixel_edges,
                                                      feedid, obsids, threshold=0.0, niter=5)
    out['destriper_offsets_niter5'] = result5
    out['destriper_map_niter5'] = maps5['map']
    meta['destriper_inputs'] = dict(n_feeds=2, n_samples=20_000, npix_side=60, offset_length=L,
                                    seed=7, sha256=[synthetic.sha256(a) for a in (pointing, tod, weights)])


def run_destriper_timing(meta, c4_npz=None):
    """The reference's CG at C4 size (19 feeds x 180,000 samples, L = 50,
    480 x 480 map) timed here for the bench line's CPU baseline: destriper_iteration with
    niter = 4 and niter = 1 (threshold 0), the difference / 3 = seconds per CG iteration
    (3 op_Ax calls each, as shipped).  c4_npz: the bench's own C4 problem (dumped on the GPU
    box by scripts/dump_c4_problem.py: read_comap_data band 0 of the reduced C2 observation),
    so the reference is timed on exactly what the GPU leg solves; without it a synthetic
    problem of 3.42 M samples (rounds 1-4)."""
    import Destriper
    L = 50
    if c4_npz:
        z = np.load(c4_npz)
        pointing, tod, weights = (np.asarray(z['pointing'], np.int64), np.asarray(z['tod'], np.float64),
                                  np.asarray(z['weights'], np.float64))
        src = f'the bench C4 problem (scripts/dump_c4_problem.py -> {os.path.basename(c4_npz)}, ' \
              f'sha256 {synthetic.sha256(tod)[:16]})'
    else:
        pointing, tod, weights = synthetic.destriper_inputs(n_feeds=19, n_samples=180_000, npix_side=480)
        src = 'synthetic.destriper_inputs(n_feeds=19, n_samples=180000, npix_side=480)'
    pixel_edges = np.arange(480 * 480)
    z = np.zeros(tod.size)
    feedid = np.repeat(np.arange(1, 20), tod.size // 19)
    obsids = np.ones(tod.size, dtype=int)
    secs = {}
    for niter in (1, 4):
        t0 = time.perf_counter()
        Destriper.destriper_iteration(pointing, z, tod, weights, L, pixel_edges, feedid, obsids, threshold=0.0,
                                      niter=niter)
        secs[niter] = time.perf_counter() - t0
    per = (secs[4] - secs[1]) / 3
    meta['reference_destriper_c4'] = {'n_samples': int(tod.size), 'n_offsets': int(tod.size // L),
                                      'iters': 3, 'seconds': secs[4] - secs[1], 'iters_per_s': 1.0 / per,
                                      'inputs': src, 'host': '8-core Xeon build container, 1 process'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--skip-l1', action='store_true')
    ap.add_argument('--only-variants', action='store_true')
    ap.add_argument('--only-comapdata', action='store_true')
    ap.add_argument('--only-binning', action='store_true')
    ap.add_argument('--only-noise', action='store_true')
    ap.add_argument('--only-variants-new', action='store_true', help='tinyscan + f3 variants only')
    ap.add_argument('--only-timing', action='store_true', help='reference destriper C4 timing only')
    ap.add_argument('--c4-npz', default=None, help='time the reference on this dumped C4 problem')
    ap.add_argument('--variants', nargs='+', default=None, help='only these Level-1 variants (variants.NAMES)')
    args = ap.parse_args()
    if args.variants:
        os.environ.setdefault('MPLBACKEND', 'agg')
        build_reference_helpers()
        install_stubs()
        figdir = os.path.join(SCRATCH, 'figures')
        os.makedirs(figdir, exist_ok=True)
        mp = os.path.join(HERE, 'golden_meta.json')
        meta = json.load(open(mp))
        for name in args.variants:
            meta[f'l1_{name}_sha256'] = run_l1_variant(name, figdir)
        json.dump(meta, open(mp, 'w'), indent=1, default=str)
        return
    if args.only_variants_new or args.only_timing:
        os.environ.setdefault('MPLBACKEND', 'agg')
        build_reference_helpers()
        install_stubs()
        mp = os.path.join(HERE, 'golden_meta.json')
        meta = json.load(open(mp))
        if args.only_variants_new:
            figdir = os.path.join(SCRATCH, 'figures')
            os.makedirs(figdir, exist_ok=True)
            for name in ('tinyscan', 'f3'):
                meta[f'l1_{name}_sha256'] = run_l1_variant(name, figdir)
        if args.only_timing:
            run_destriper_timing(meta, args.c4_npz)
        json.dump(meta, open(mp, 'w'), indent=1, default=str)
        return
    if args.only_noise:
        os.environ.setdefault('MPLBACKEND', 'agg')
        build_reference_helpers()
        install_stubs()
        mp = os.path.join(HERE, 'golden_meta.json')
        meta = json.load(open(mp))
        meta['reference_timings_s_noise'] = run_noise()
        json.dump(meta, open(mp, 'w'), indent=1, default=str)
        return
    if args.only_binning:
        os.environ.setdefault('MPLBACKEND', 'agg')
        build_reference_helpers()
        install_stubs()
        run_binning()
        return
    if args.only_comapdata:
        build_reference_helpers()
        install_stubs()
        mp = os.path.join(HERE, 'golden_meta.json')
        meta = json.load(open(mp))
        meta['comapdata_sha256'] = run_comapdata()
        meta['parser_case'] = run_parser()
        json.dump(meta, open(mp, 'w'), indent=1, default=str)
        return
    if args.only_variants:
        os.environ.setdefault('MPLBACKEND', 'agg')
        build_reference_helpers()
        install_stubs()
        figdir = os.path.join(SCRATCH, 'figures')
        os.makedirs(figdir, exist_ok=True)
        import variants
        mp = os.path.join(HERE, 'golden_meta.json')
        meta = json.load(open(mp))
        for name in variants.NAMES:
            meta[f'l1_{name}_sha256'] = run_l1_variant(name, figdir)
        run_spikes()
        json.dump(meta, open(mp, 'w'), indent=1, default=str)
        return
    os.environ.setdefault('MPLBACKEND', 'agg')
    build_reference_helpers()
    install_stubs()
    figdir = os.path.join(SCRATCH, 'figures')
    os.makedirs(figdir, exist_ok=True)
    meta = {'reference': 'SharperJBCA/COMAPreduce comancpipeline/version.py __version__ 0.9.1',
            'generated_by': 'tests/golden/make_golden.py', 'numpy': np.__version__}
    mf, bv, ds = {}, {}, {}
    run_medfilt(mf)
    meta['medfilt_cases'] = MEDFILT_CASES
    run_binvalues(bv)
    run_destriper(ds, meta)
    np.savez_compressed(os.path.join(HERE, 'golden_medfilt.npz'), **mf)
    np.savez_compressed(os.path.join(HERE, 'golden_binvalues.npz'), **bv)
    np.savez_compressed(os.path.join(HERE, 'golden_destriper.npz'), **ds)
    if not args.skip_l1:
        l1 = {}
        run_l1(l1, meta, figdir)
        np.savez_compressed(os.path.join(HERE, 'golden_l1_c1.npz'), **l1)
    old = {}
    mp = os.path.join(HERE, 'golden_meta.json')
    if os.path.exists(mp):
        old = json.load(open(mp))
    old.update(meta)
    json.dump(old, open(mp, 'w'), indent=1, default=str)
    print(json.dumps(meta, indent=1, default=str))


if __name__ == '__main__':
    main()
