"""Destriper data prep (COMAPData.read_comap_data) against
the reference's own outputs (tests/golden/golden_comapdata.npz, made by
make_golden.py --only-comapdata running the reference COMAPData module).

The astrometric leaves (WCS, healpy Rotator, get_sun) are this repo's
restatements on both sides, so these tests pin everything downstream of
them; the leaves themselves are parity-unpinned."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, 'golden'))
import comapdata_case as cc  # noqa: E402

from comapreduce_amd.mapmaking import comapdata as cd  # noqa: E402
from comapreduce_amd.mapmaking.wcs import CelestialWCS  # noqa: E402


@pytest.fixture(scope='module')
def case_store():
    return cc.store()


@pytest.fixture(scope='module')
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, 'golden_comapdata.npz'))


def map_info(m):
    return cd.map_info_from(m['crval'], m['cdelt'], m['crpix'], m['ctype'], m['nxpix'], m['nypix'])


def check_outputs(res, golden, name, exact_tod=True):
    for k, v in zip(cc.OUTPUTS, res):
        v = np.asarray(v)
        if k in cc.STRIDED:
            v = v[::cc.STRIDE]
        g = golden[f'{name}__{k}']
        assert v.shape == g.shape, (name, k, v.shape, g.shape)
        if k in ('pointing', 'remapping_array', 'feedid', 'obsids', 'weights') or exact_tod:
            assert np.array_equal(v, g), (name, k)
        else:
            assert np.max(np.abs(v - g)) <= 1e-12 * max(np.max(np.abs(g)), 1.0), (name, k)


def test_fixture_inputs_reproducible(case_store, golden_dir):
    import json
    meta = json.load(open(os.path.join(golden_dir, 'golden_meta.json')))['comapdata_sha256']
    from comapreduce_amd import synthetic
    store, names = case_store
    for n in names:
        for k, v in store[n][0].items():
            assert synthetic.sha256(np.asarray(v)) == meta[n][k], (n, k)


@pytest.mark.parametrize('name', list(cc.CASES))
def test_oracle_comapdata_matches_reference(case_store, golden, name):
    from oracle import comapdata as oc
    store, names = case_store
    case = cc.CASES[name]
    res = oc.read_comap_data(names, store, map_info(case['map']), feeds=cc.FEEDS, **case['kw'])
    check_outputs(res, golden, name)


@pytest.mark.parametrize('name', list(cc.CASES))
def test_host_prep_matches_reference_with_checker_median(case_store, golden, name, monkeypatch):
    """Host logic of the product prep; the device median call is replaced by
    the oracle (medianFilter.cpp restatement) so this runs without a GPU."""
    import oracle
    from comapreduce_amd.tools import medfilt as mf

    def checker(series, w, reflect=False, device=None):
        out = []
        for s in series:
            z = np.concatenate((s[::-1], s, s[::-1])) if reflect else s.copy()
            y = oracle.medfilt(z.astype(np.float64), int(w))
            out.append(y[s.size:2 * s.size] if reflect else y)
        return out
    monkeypatch.setattr(mf, 'medfilt_batch', checker)
    store, names = case_store
    case = cc.CASES[name]
    res = cd.read_comap_data(names, map_info(case['map']), feeds=cc.FEEDS, store=store, **case['kw'])
    check_outputs(res, golden, name)


@pytest.mark.gpu
@pytest.mark.parametrize('name', list(cc.CASES))
def test_gpu_prep_matches_reference(case_store, golden, name):
    store, names = case_store
    case = cc.CASES[name]
    res = cd.read_comap_data(names, map_info(case['map']), feeds=cc.FEEDS, store=store, **case['kw'])
    check_outputs(res, golden, name)


@pytest.mark.gpu
def test_gpu_medfilt_batch_reflect_bit_exact():
    import oracle
    from comapreduce_amd.tools.medfilt import medfilt_batch
    rng = np.random.default_rng(4)
    series = [np.round(rng.standard_normal(n), 2) for n in (801, 400, 5000, 12345, 2000)]
    for reflect in (False, True):
        got = medfilt_batch(series, 400, reflect=reflect)
        for s, g in zip(series, got):
            z = np.concatenate((s[::-1], s, s[::-1])) if reflect else s.copy()
            y = oracle.medfilt(z, 400)
            assert np.array_equal(g, y[s.size:2 * s.size] if reflect else y), (s.size, reflect)


def test_parse_bit_mask_and_getfeeds_match_oracle():
    from oracle import comapdata as oc
    for flag in [0, 1, 2, 5, 32, 33, 36, 255, 1024 + 32, 2 ** 20 + 1]:
        assert cd.parse_bit_mask(flag) == oc.parse_bit_mask(flag), flag
    rng = np.random.default_rng(3)
    for _ in range(50):
        ff = np.sort(rng.choice(np.arange(1, 21), rng.integers(1, 20), replace=False))
        sel = np.sort(rng.choice(np.arange(1, 21), rng.integers(1, 20), replace=False))
        a, b = cd.GetFeeds(ff, sel), oc.get_feeds(ff, sel)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_wcs_reference_pixel_and_symmetry():
    for proj in ('CAR', 'SIN', 'TAN'):
        w = CelestialWCS([83.6, 22.0], [-0.01, 0.01], [101, 51], [f'RA---{proj}', f'DEC--{proj}'])
        px, py = w.wcs_world2pix(np.array([83.6]), np.array([22.0]), 0)
        assert abs(px[0] - 100) < 1e-9 and abs(py[0] - 50) < 1e-9, proj
        # east is to the left for negative CDELT1; north is up
        px2, py2 = w.wcs_world2pix(np.array([83.7]), np.array([22.1]), 0)
        assert px2[0] < 100 and py2[0] > 50, proj
    # CAR on the equator is the plate carree grid
    w = CelestialWCS([10.0, 0.0], [-0.5, 0.5], [1, 1], ['RA---CAR', 'DEC--CAR'])
    px, py = w.wcs_world2pix(np.array([9.0, 11.0]), np.array([1.0, -2.0]), 0)
    assert np.allclose(px, [2.0, -2.0]) and np.allclose(py, [2.0, -4.0])


def test_transform_to_1d_offmap():
    from comapreduce_amd.mapmaking.wcs import transform_to_1d
    w = CelestialWCS([10.0, 0.0], [-1.0, 1.0], [3, 3], ['RA---CAR', 'DEC--CAR'])
    idx = transform_to_1d(np.array([10.0, 20.0, 10.0, 9.0]), np.array([0.0, 0.0, 5.0, 1.0]), w, 5, 5)
    assert idx.tolist() == [2 * 5 + 2, -1, -1, 3 * 5 + 3]


def test_read_comap_data_bands_equals_per_band(case_store, monkeypatch):
    """read_comap_data_bands (one call for all bands, the batched destriper's
    input) restricted to band b's kept offsets == read_comap_data(iband=b)."""
    import oracle
    from comapreduce_amd.tools import medfilt as mf

    def checker(series, w, reflect=False, device=None):
        out = []
        for s in series:
            z = np.concatenate((s[::-1], s, s[::-1])) if reflect else s.copy()
            y = oracle.medfilt(z.astype(np.float64), int(w))
            out.append(y[s.size:2 * s.size] if reflect else y)
        return out
    monkeypatch.setattr(mf, 'medfilt_batch', checker)
    store, names = case_store
    case = cc.CASES['car']
    kw = {k: v for k, v in case['kw'].items() if k != 'iband'}
    r = cd.read_comap_data_bands(names, map_info(case['map']), bands=(0, 1, 2, 3), feeds=cc.FEEDS, store=store, **kw)
    L = kw.get('offset_length', 50)
    assert r['tod'].shape[0] == 4 and r['keep'].shape == (4, r['pointing'].size // L)
    for b in range(4):
        one = cd.read_comap_data(names, map_info(case['map']), feeds=cc.FEEDS, store=store, iband=b, **kw)
        sel = np.repeat(r['keep'][b].astype(bool), L)
        for k, v in (('tod', r['tod'][b]), ('weights', r['weights'][b]), ('pointing', r['pointing']),
                     ('az', r['az']), ('feedid', r['feedid']), ('obsids', r['obsids'])):
            i = cc.OUTPUTS.index(k)
            assert np.array_equal(v[sel], one[i]), (b, k)
        # dropped offsets carry no weight in that band
        assert not r['weights'][b][~sel].any()


def test_nan_samples_do_not_abort_prep(case_store, monkeypatch):
    """A non-finite Level-2 sample (e.g. a zero vane gain upstream) is left out of
    the 400-sample median input instead of aborting the run; it ends with tod 0 and
    weight 0 as in the reference (COMAPData.py:550-552)."""
    import oracle
    from comapreduce_amd.tools import medfilt as mf
    seen = []

    def checker(series, w, reflect=False, device=None):
        out = []
        for s in series:
            assert np.isfinite(s).all()
            seen.append(s.size)
            z = np.concatenate((s[::-1], s, s[::-1])) if reflect else s.copy()
            y = oracle.medfilt(z.astype(np.float64), int(w))
            out.append(y[s.size:2 * s.size] if reflect else y)
        return out
    monkeypatch.setattr(mf, 'medfilt_batch', checker)
    store, names = case_store
    ds, attrs = store[names[1]]
    ds = dict(ds)
    tod = ds['averaged_tod/tod'].copy()
    s0, e0 = ds['averaged_tod/scan_edges'][0]
    tod[0, 0, s0 + 2500:s0 + 2510] = np.nan
    ds['averaged_tod/tod'] = tod
    st = dict(store)
    st[names[1]] = (ds, attrs)
    case = cc.CASES['car']
    res = cd.read_comap_data([names[1]], map_info(case['map']), feeds=cc.FEEDS, store=st, **case['kw'])
    t, w = res[0], res[1]
    assert np.isfinite(t).all() and np.isfinite(w).all()
    assert seen
