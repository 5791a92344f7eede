"""Destriper data prep (COMAPData.read_comap_data) against
the reference's own outputs (tests/golden/golden_comapdata.npz, made by
make_golden.py --only-comapdata running the reference COMAPData module).

The astrometric leaves (WCS, healpy Rotator, get_sun) are this repo's
restatements on both sides, so these tests pin everything downstream of
them; the WCS and Sun leaves are pinned to astropy 4.3.1 separately
(tests/test_astro_golden.py), healpy's Rotator / ang2pix stay unpinned
(healpy is absent from the image)."""
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


# the Sun-centric distance / colatitude are trigonometric leaves: the device's f64 libm
# sits within an ulp or two of NumPy's, every other output is exact
TRIG = ('ra', 'dec')


def check_outputs(res, golden, name, device=False):
    for k, v in zip(cc.OUTPUTS, res):
        v = np.asarray(v)
        if k in cc.STRIDED:
            v = v[::cc.STRIDE]
        g = golden[f'{name}__{k}']
        assert v.shape == g.shape, (name, k, v.shape, g.shape)
        if device and k in TRIG:
            assert np.max(np.abs(v - g)) <= 1e-12 * max(np.max(np.abs(g)), 1.0), (name, k)
        else:
            assert np.array_equal(v, g), (name, k)


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


@pytest.mark.gpu
@pytest.mark.parametrize('name', list(cc.CASES))
def test_gpu_prep_matches_reference(case_store, golden, name):
    store, names = case_store
    case = cc.CASES[name]
    res = cd.read_comap_data(names, map_info(case['map']), feeds=cc.FEEDS, store=store, **case['kw'])
    check_outputs(res, golden, name, device=True)


@pytest.mark.gpu
@pytest.mark.parametrize('name', list(cc.CASES))
def test_gpu_prep_device_inputs_and_outputs(case_store, golden, name):
    """The in-memory chain's form: Level-2 datasets already on the device (torch
    tensors, as the L1 -> L2 stages leave them) and device outputs -- the same
    vectors as from host arrays."""
    import torch
    store, names = case_store
    dstore = {fn: ({k: (torch.as_tensor(v, device='cuda') if isinstance(v, np.ndarray) and v.dtype != object
                        else v) for k, v in ds.items()}, at) for fn, (ds, at) in store.items()}
    case = cc.CASES[name]
    res = cd.read_comap_data(names, map_info(case['map']), feeds=cc.FEEDS, store=dstore, device_outputs=True,
                             **case['kw'])
    assert all(isinstance(v, torch.Tensor) for i, v in enumerate(res) if cc.OUTPUTS[i] != 'remapping_array')
    check_outputs([v.cpu().numpy() if hasattr(v, 'cpu') else v for v in res], golden, name, device=True)


@pytest.mark.gpu
def test_gpu_prep_pieces_vs_numpy():
    """The device auto_rms (NumPy's pairwise nanstd tree, NaNs included) and the az / el
    percentiles (exact order statistics + NumPy's linear rule, ties included) equal
    NumPy bit for bit on rows of many lengths."""
    import torch
    from comapreduce_amd import _native as N
    c = N.ctx(0)
    N.bind_stream(c, torch.device('cuda', 0))
    rng = np.random.default_rng(8)
    for T in (3, 9, 130, 1001, 8193, 16386, 40001, 180000):
        x = (rng.standard_normal((4, T)) * 3 + 7) / 1.7
        x[1, rng.random(T) < 0.3] = 0.0
        x[2, rng.random(T) < 0.05] = np.nan
        x[3] = np.round(x[3], 1)
        scale = np.array([1.0, 1.37, 0.9, 2.5])
        # (every device operand is held by a name until the call has run: a temporary's
        # memory could be handed to the next temporary before the kernel reads it)
        xd, sd = torch.as_tensor(x, device='cuda'), torch.as_tensor(scale, device='cuda')
        rows = torch.arange(4, dtype=torch.int32, device='cuda')
        out = torch.empty(4, dtype=torch.float64, device='cuda')
        N.check(N.lib().comap_prep_auto_rms(c, N.dptr(xd), T, N.dptr(rows), N.dptr(sd), 4, T, N.dptr(out)), c,
                'auto_rms')
        for r in range(4):
            want = cd.auto_rms(x[r] / scale[r])
            got = out[r].item()
            assert (np.isnan(want) and np.isnan(got)) or want == got, (T, r, want, got)
        az = np.round(rng.standard_normal((3, T)) * 20 + 180, 2)
        az[1, rng.random(T) < 0.1] = np.nan
        az[0] = np.round(rng.standard_normal(T) * 2, 1)          # both signs, zeros, -0.0, ties
        az[0, rng.random(T) < 0.05] = -0.0
        el = np.round(rng.standard_normal((3, T)) * 5 + 45, 3)
        el[2, 0] = np.nan if T > 3 else el[2, 0]
        pct = torch.empty((3, 4), dtype=torch.float64, device='cuda')
        r3 = torch.arange(3, dtype=torch.int32, device='cuda')
        azd, eld = torch.as_tensor(az, device='cuda'), torch.as_tensor(el, device='cuda')
        N.check(N.lib().comap_prep_percentiles(c, N.dptr(azd), N.dptr(eld), T, N.dptr(r3), 3, T, N.dptr(pct)), c,
                'percentiles')
        p = pct.cpu().numpy()
        for r in range(3):
            g = np.isfinite(az[r])
            want = [np.percentile(az[r][g], 10), np.percentile(az[r][g], 90), np.percentile(el[r][g], 10),
                    np.percentile(el[r][g], 90)]
            assert np.array_equal(p[r], want, equal_nan=True), (T, r, p[r], want)


@pytest.mark.gpu
@pytest.mark.parametrize('w', [400, 401, 64])
def test_gpu_highpass_vs_reference_medfilt(w):
    """comap_prep_highpass on segments with zeros (compacted away), -0.0, ties and
    lengths from just above 2w to many windows: every non-zero sample minus the
    reference's reflect-padded medfilt of its segment's non-zero samples, zeros kept."""
    import torch
    import oracle
    from comapreduce_amd import _native as N
    c = N.ctx(0)
    N.bind_stream(c, torch.device('cuda', 0))
    rng = np.random.default_rng(w)
    lens = [2 * w + 1, 2 * w + 7, 3000, 1000, 17000]
    x = np.concatenate([np.round(rng.standard_normal(n) * 4, 1) for n in lens])
    x[rng.random(x.size) < 0.1] = 0.0
    x[rng.random(x.size) < 0.01] = -0.0
    starts = np.concatenate(([0], np.cumsum(lens)[:-1]))
    segs = np.stack([starts, np.asarray(lens)], axis=1).astype(np.int64)
    sd = torch.as_tensor(segs, device='cuda')
    xd = torch.as_tensor(x, device='cuda')
    N.check(N.lib().comap_prep_highpass(c, N.dptr(xd), N.dptr(sd), len(lens), w), c, 'highpass')
    got = xd.cpu().numpy()
    for s0, n in segs:
        seg = x[s0:s0 + n]
        nz = seg != 0
        v = seg[nz]
        if v.size <= 2 * w:
            continue
        z = np.concatenate((v[::-1], v, v[::-1]))
        want = seg.copy()
        want[nz] = v - oracle.medfilt(z, w)[v.size:2 * v.size]
        assert np.array_equal(got[s0:s0 + n], want), (w, s0, n)


@pytest.mark.gpu
def test_gpu_highpass_nonfinite_vs_reference():
    """COMAPData.median_filter on non-zero samples that include +-inf and NaN
    (COMAPData.py:72-81, 357-360): +-inf stays in the running median's input (single
    samples, runs that make window medians +-inf, windows whose middle pair is -inf / +inf
    -> NaN); short segments (<= 2w non-zero values, NaN included) get np.nanmedian of
    the non-NaN values; NaN samples stay NaN.  Checked against oracle.medfilt, which
    test_oracle_golden pins to the reference's compiled filter on +-inf input.  (Long
    segments holding NaN are unpinned, DESIGN.md §9, and are not in this fixture.)"""
    import torch
    import oracle
    from comapreduce_amd import _native as N
    c = N.ctx(0)
    N.bind_stream(c, torch.device('cuda', 0))
    w = 400
    rng = np.random.default_rng(77)
    lens = [3000, 2 * w + 3, 5000, 500, 700, 120, 4000]
    parts = []
    for k, n in enumerate(lens):
        v = np.round(rng.standard_normal(n) * 4, 1)
        v[rng.random(n) < 0.1] = 0.0
        if n > 2 * w:                                   # running median: +-inf only
            v[rng.random(n) < 0.02] = np.inf
            v[rng.random(n) < 0.02] = -np.inf
            if k == 2:
                v[1000:1250] = np.inf                   # window medians +inf
                v[1250:1500] = -np.inf                  # middle pair -inf / +inf -> NaN
        else:                                           # np.nanmedian: NaN and +-inf
            v[rng.random(n) < 0.15] = np.nan
            v[3] = np.inf
            if k == 5:
                v[:] = np.nan                           # all NaN: nanmedian NaN
        parts.append(v)
    x = np.concatenate(parts)
    starts = np.concatenate(([0], np.cumsum(lens)[:-1]))
    segs = np.stack([starts, np.asarray(lens)], axis=1).astype(np.int64)
    sd = torch.as_tensor(segs, device='cuda')
    xd = torch.as_tensor(x, device='cuda')
    N.check(N.lib().comap_prep_highpass(c, N.dptr(xd), N.dptr(sd), len(lens), w), c, 'highpass')
    got = xd.cpu().numpy()
    with np.errstate(invalid='ignore'):
        for s0, n in segs:
            seg = x[s0:s0 + n]
            nz = seg != 0
            v = seg[nz]
            if v.size > 2 * w:
                z = np.concatenate((v[::-1], v, v[::-1]))
                f = oracle.medfilt(z, w)[v.size:2 * v.size]
            else:
                f = np.ones(v.size) * (np.nanmedian(v) if (~np.isnan(v)).any() else np.nan)
            want = seg.copy()
            want[nz] = v - f
            assert np.array_equal(got[s0:s0 + n], want, equal_nan=True), (s0, n)
            if v.size > 2 * w:
                assert np.isinf(f).any() or n != 5000


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


@pytest.mark.gpu
def test_read_comap_data_bands_equals_per_band(case_store):
    """read_comap_data_bands (one call for all bands, the batched destriper's
    input) restricted to band b's kept offsets == read_comap_data(iband=b)."""
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


@pytest.mark.gpu
@pytest.mark.parametrize('where', ['burst', 'scattered', 'head_tail', 'short_segment'])
def test_nan_samples_prep_vs_reference_semantics(case_store, where):
    """NaN Level-2 samples (e.g. a zero vane gain upstream) stay in the high-pass median
    input as in the reference (bad = tod == 0, COMAPData.py:357-360): a segment of > 2 x 400
    values goes through the reference's two-heap running median, whose result for NaN
    follows its insertion history (Mediator.h), a shorter one through np.nanmedian (:79).
    The device (two-heap replay for NaN-bearing segments) equals the oracle's prep, whose
    medfilt is the two-heap restatement pinned against the reference's compiled filter
    (tests/test_oracle_golden.py), bit for bit; NaN samples end with tod 0 and weight 0
    (COMAPData.py:550-552)."""
    store, names = case_store
    ds, attrs = store[names[1]]
    ds = dict(ds)
    tod = ds['averaged_tod/tod'].copy()
    edges = ds['averaged_tod/scan_edges']
    s0, e0 = edges[0]
    if where == 'burst':
        tod[0, 0, s0 + 2500:s0 + 2510] = np.nan
        tod[0, 3, s0 + 5000:s0 + 5300] = np.nan      # longer than w/2: NaN-dominated windows
    elif where == 'scattered':
        rng = np.random.default_rng(7)
        idx = s0 + rng.choice(e0 - s0, 40, replace=False)
        tod[0, 0, idx] = np.nan
        tod[1, 2, idx[:5]] = np.nan
    elif where == 'head_tail':
        tod[0, 1, s0:s0 + 3] = np.nan
        tod[0, 1, e0 - 60:e0] = np.nan
    else:
        # a scan re-cut to 600 samples (<= 2w values: np.nanmedian ignores NaN)
        edges = edges.copy()
        edges[0, 1] = edges[0, 0] + 600
        ds['averaged_tod/scan_edges'] = edges
        tod[0, 0, s0 + 100:s0 + 104] = np.nan
    ds['averaged_tod/tod'] = tod
    st = dict(store)
    st[names[1]] = (ds, attrs)
    case = cc.CASES['car']
    res = cd.read_comap_data([names[1]], map_info(case['map']), feeds=cc.FEEDS, store=st, **case['kw'])
    t, w = res[0], res[1]
    assert np.isfinite(t).all() and np.isfinite(w).all()
    from oracle import comapdata as oc
    ref = oc.read_comap_data([names[1]], st, map_info(case['map']), feeds=cc.FEEDS, **case['kw'])
    for k, a, b in zip(cc.OUTPUTS, res, ref):
        a, b = np.asarray(a), np.asarray(b)
        if k in TRIG:
            assert np.max(np.abs(a - b)) <= 1e-12 * max(np.max(np.abs(b)), 1.0), k
        else:
            assert np.array_equal(a, b), k


def _many_scans_store(case_store, dense=False):
    """File 13 of the golden scenario re-cut into 82 scans (> the 64 a scan table once
    held): lengths cycle through 30 (shorter than L: no samples), 120 / 260 / 75 / 240
    (short segments, np.nanmedian) and 900 (> 2 x 400: the running median).  dense: more
    than 128 scans (the gather kernel's in-LDS scan table holds 128; beyond it the table is
    binary-searched in HBM) -- shorter cycles, 5-sample gaps."""
    store, names = case_store
    ds, attrs = store[names[1]]
    ds = dict(ds)
    T = ds['averaged_tod/tod'].shape[-1]
    edges, t = [], 100
    cyc = (30, 60, 100, 75, 90, 45, 55, 65, 820) if dense else (30, 120, 260, 900, 75, 240)
    gap = 5 if dense else 20
    while True:
        n = cyc[len(edges) % len(cyc)]
        if t + n > T:
            break
        edges.append((t, t + n))
        t += n + gap
    ds['averaged_tod/scan_edges'] = np.asarray(edges, dtype=np.int64)
    return {names[1]: (ds, attrs)}, [names[1]], len(edges)


@pytest.mark.gpu
@pytest.mark.parametrize('dense', [False, True])
@pytest.mark.parametrize('name', list(cc.CASES))
def test_gpu_prep_many_scans_vs_oracle(case_store, name, dense):
    """read_comap_data on a file of 82 (dense: > 128, the HBM-searched scan table) scans
    (COMAPData.py:350-360 loops over any number) == the oracle, bit for bit except the
    Sun-centric trigonometric leaves."""
    from oracle import comapdata as oc
    store, names, S = _many_scans_store(case_store, dense)
    assert S > (128 if dense else 64), S
    case = cc.CASES[name]
    ref = oc.read_comap_data(names, store, map_info(case['map']), feeds=cc.FEEDS, **case['kw'])
    got = cd.read_comap_data(names, map_info(case['map']), feeds=cc.FEEDS, store=store, **case['kw'])
    for k, a, b in zip(cc.OUTPUTS, got, ref):
        a, b = np.asarray(a), np.asarray(b)
        assert a.shape == b.shape, k
        if k in TRIG:
            assert np.max(np.abs(a - b)) <= 1e-12 * max(np.max(np.abs(b)), 1.0), k
        else:
            assert np.array_equal(a, b), k


@pytest.mark.gpu
def test_gpu_prep_selected_feeds_missing_from_file(case_store):
    """A feed selection wider than a file's feeds (countDataSize sizes the arrays for every
    selected feed, the file fills only the rows it holds): the unfilled tail is zeros and
    cut like the reference's, so the outputs equal the oracle's (an uninitialised tail
    once reached the map binning as garbage pixel ids)."""
    from oracle import comapdata as oc
    store, names = case_store
    case = cc.CASES[list(cc.CASES)[0]]
    feeds = list(cc.FEEDS) + [f for f in range(1, 20) if f not in cc.FEEDS][:3]
    ref = oc.read_comap_data(names, store, map_info(case['map']), feeds=feeds, **case['kw'])
    got = cd.read_comap_data(names, map_info(case['map']), feeds=feeds, store=store, **case['kw'])
    for k, a, b in zip(cc.OUTPUTS, got, ref):
        a, b = np.asarray(a), np.asarray(b)
        assert a.shape == b.shape, k
        if k in TRIG:
            assert np.max(np.abs(a - b)) <= 1e-12 * max(np.max(np.abs(b)), 1.0), k
        else:
            assert np.array_equal(a, b), k


def _nonfinite_store(case_store):
    """The 82-scan file with +-inf samples inside 900-sample scans (the running median
    over > 2 x 400 values: the reference keeps +-inf in its input, bad = tod == 0,
    COMAPData.py:357-360) of file feed 0, and NaN inside 120- and 260-sample scans
    (np.nanmedian, :79: NaN ignored) of file feed 2.  +-inf makes feed 0's auto_rms weight
    non-finite, so the cut drops its offsets (:550-557); NaN leaves feed 2's weight finite
    and its short scans visible.  medfilt_batch pins +-inf inside the running median
    itself (test_gpu_l1.py::test_medfilt_dropin_infinities)."""
    store, names, S = _many_scans_store(case_store)
    ds, attrs = store[names[0]]
    ds = dict(ds)
    tod = ds['averaged_tod/tod'].copy()
    edges = ds['averaged_tod/scan_edges']
    lengths = edges[:, 1] - edges[:, 0]
    longs = edges[lengths == 900]
    shorts = edges[(lengths == 120) | (lengths == 260)]
    assert len(longs) >= 3 and len(shorts) >= 4
    for k, (s, e) in enumerate(longs[:3]):
        tod[0, :, s + 300 + 7 * k] = np.inf
        tod[0, :, s + 420:s + 426] = np.inf                 # a run: shifts the order by 6
        tod[0, :, s + 610 + k] = -np.inf
    for k, (s, e) in enumerate(shorts[:4]):
        tod[2, :, s + 10 + k] = np.nan
        tod[2, :, s + 40:s + 44] = np.nan
    ds['averaged_tod/tod'] = tod
    return {names[0]: (ds, attrs)}, names


def test_oracle_nonfinite_prep_runs(case_store):
    """The oracle runs the +-inf / NaN fixture, and its running median (oracle.medfilt)
    equals the reference's compiled filter on series holding +-inf (test_oracle_golden
    pins that directly)."""
    from oracle import comapdata as oc
    store, names = _nonfinite_store(case_store)
    case = cc.CASES['car']
    res = oc.read_comap_data(names, store, map_info(case['map']), feeds=cc.FEEDS, **case['kw'])
    assert np.isfinite(res[0]).all() and np.isfinite(res[1]).all() and res[0].size > 0


@pytest.mark.gpu
@pytest.mark.parametrize('name', list(cc.CASES))
def test_gpu_prep_nonfinite_vs_oracle(case_store, name):
    """+-inf samples stay in the 400-sample running-median input and NaN drops out of
    the short scans' np.nanmedian, as in the reference (COMAPData.py:72-81, 357-360):
    read_comap_data == the oracle bit for bit (Sun-centric trigonometric leaves aside)."""
    from oracle import comapdata as oc
    store, names = _nonfinite_store(case_store)
    case = cc.CASES[name]
    ref = oc.read_comap_data(names, store, map_info(case['map']), feeds=cc.FEEDS, **case['kw'])
    got = cd.read_comap_data(names, map_info(case['map']), feeds=cc.FEEDS, store=store, **case['kw'])
    for k, a, b in zip(cc.OUTPUTS, got, ref):
        a, b = np.asarray(a), np.asarray(b)
        assert a.shape == b.shape, k
        if k in TRIG:
            assert np.max(np.abs(a - b)) <= 1e-12 * max(np.max(np.abs(b)), 1.0), k
        else:
            assert np.array_equal(a, b), k


def test_oracle_many_scans_runs(case_store):
    """The many-scan fixture is a real case for the oracle: several scans of each kind."""
    from oracle import comapdata as oc
    store, names, S = _many_scans_store(case_store)
    case = cc.CASES['car']
    res = oc.read_comap_data(names, store, map_info(case['map']), feeds=cc.FEEDS, **case['kw'])
    assert S > 64 and res[0].size > 0 and res[0].size % 50 == 0


def test_lazy_outputs_resolve_on_every_read_path():
    """read_comap_data_bands' one-rank device-output dict forms remapping_array on first
    read; dict(r), {**r}, copy, pop, iteration and pickling must all see the value,
    never a placeholder."""
    import pickle
    from comapreduce_amd.mapmaking.comapdata import _LazyOutputs

    def make(v):
        r = _LazyOutputs({'tod': 1})
        r.lazy('remapping_array', lambda: v)
        return r
    assert dict(make(1))['remapping_array'] == 1
    assert {**make(2)}['remapping_array'] == 2
    assert make(3).copy()['remapping_array'] == 3
    assert make(4).pop('remapping_array') == 4
    assert pickle.loads(pickle.dumps(make(5)))['remapping_array'] == 5
    assert [make(6)[k] for k in make(6)] == [1, 6]
    assert dict(make(7).items())['remapping_array'] == 7
