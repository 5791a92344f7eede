"""Pins the CPU oracle to the reference's own outputs (tests/golden, made by
tests/golden/make_golden.py running COMAPreduce v0.9.1 in the build container)."""
import json
import os

import numpy as np
import pytest

import oracle
from oracle import l1 as ol1
from comapreduce_amd import synthetic


def meta(golden_dir):
    return json.load(open(os.path.join(golden_dir, 'golden_meta.json')))


def relmax(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin), 'NaN pattern differs'
    return np.max(np.abs(a[fin] - b[fin])) / max(np.max(np.abs(b[fin])), 1e-300)


def test_medfilt_oracle_bit_exact(golden_dir):
    g = np.load(os.path.join(golden_dir, 'golden_medfilt.npz'))
    for seed, n, w in meta(golden_dir)['medfilt_cases']:
        x = np.random.default_rng(seed).standard_normal(n)
        assert np.array_equal(oracle.medfilt(x.copy(), w), g[f'medfilt_{seed}_{n}_{w}']), (seed, n, w)


def test_medfilt_reference_build_matches_golden(golden_dir):
    if oracle.ref_lib() is None:
        pytest.skip('oracle/_ref not built (reference sources absent)')
    g = np.load(os.path.join(golden_dir, 'golden_medfilt.npz'))
    for seed, n, w in meta(golden_dir)['medfilt_cases']:
        x = np.random.default_rng(seed).standard_normal(n)
        assert np.array_equal(oracle.medfilt_reference(x.copy(), w), g[f'medfilt_{seed}_{n}_{w}'])


def test_medfilt_oracle_vs_reference_random():
    if oracle.ref_lib() is None:
        pytest.skip('oracle/_ref not built')
    rng = np.random.default_rng(5)
    for n, w in [(3000, 6), (2500, 401), (1000, 3), (7000, 2000)]:
        x = np.round(rng.standard_normal(n), 1)     # many ties
        assert np.array_equal(oracle.medfilt(x.copy(), w), oracle.medfilt_reference(x.copy(), w))


def test_medfilt_oracle_vs_reference_infinities():
    """+-inf samples (scattered, a run making window medians +inf, a run whose windows'
    middle pair is -inf / +inf): the order-statistics oracle == the reference's compiled
    two-heap filter, NaN results included."""
    if oracle.ref_lib() is None:
        pytest.skip('oracle/_ref not built')
    rng = np.random.default_rng(31)
    for n, w in [(5000, 400), (4000, 401), (3000, 6), (9000, 6000), (2000, 1)]:
        x = np.round(rng.standard_normal(n), 1)
        x[rng.random(n) < 0.03] = np.inf
        x[rng.random(n) < 0.03] = -np.inf
        a = n // 3
        x[a:a + 300] = np.inf
        x[a + 300:a + 600] = -np.inf
        want = oracle.medfilt_reference(x.copy(), w)
        got = oracle.medfilt(x.copy(), w)
        assert np.array_equal(got, want, equal_nan=True), (n, w)
        if w <= 401:                               # the 300-runs dominate these windows
            assert np.isinf(want).any() and (w % 2 or np.isnan(want).any()), (n, w)


def _nan_cases(golden_dir):
    g = np.load(os.path.join(golden_dir, 'golden_medfilt_nan.npz'))
    names = sorted(k[2:] for k in g.files if k.startswith('x_'))
    return g, names


def test_medfilt_twoheap_vs_nan_fixtures(golden_dir):
    """The two-heap restatement (oracle.medfilt on NaN input) == the reference's compiled
    filter on the committed NaN known-answer fixtures (tests/golden/make_medfilt_nan.py):
    single NaN, runs, head / tail, NaN-dominated windows, all NaN, +-inf mixed in, even /
    odd w = 1 ... 6000, series shorter than the window, reflect-padded form."""
    g, names = _nan_cases(golden_dir)
    assert len(names) == 12
    for name in names:
        x, y, w, r = g[f'x_{name}'], g[f'y_{name}'], int(g[f'w_{name}']), bool(g[f'r_{name}'])
        if r:
            z = np.concatenate((x[::-1], x, x[::-1]))
            got = oracle.medfilt(z, w)[x.size:2 * x.size]
        else:
            got = oracle.medfilt(x.copy(), w)
        assert np.array_equal(got, y, equal_nan=True), name


def test_medfilt_twoheap_vs_reference_random():
    """Random NaN / +-inf / n < w series: the two-heap restatement == oracle/_ref."""
    if oracle.ref_lib() is None:
        pytest.skip('oracle/_ref not built')
    rng = np.random.default_rng(77)
    for _ in range(150):
        n = int(rng.integers(1, 2500))
        w = int(rng.integers(1, 700))
        if n < w // 2 + w % 2:
            continue
        x = np.round(rng.standard_normal(n), 1)
        x[rng.random(n) < rng.choice([0.0, 0.01, 0.2])] = np.nan
        x[rng.random(n) < 0.01] = rng.choice([np.inf, -np.inf])
        want = oracle.medfilt_reference(x.copy(), w)
        assert np.array_equal(oracle.medfilt_twoheap(x.copy(), w), want, equal_nan=True), (n, w)
        assert np.array_equal(oracle.medfilt(x.copy(), w), want, equal_nan=True), (n, w)


def test_binvalues_oracle_bit_exact(golden_dir):
    b = np.load(os.path.join(golden_dir, 'golden_binvalues.npz'))
    rng = np.random.default_rng(21)
    npix = 1000
    pix = rng.integers(-50, npix + 50, 50_000).astype(np.int64)
    w = rng.standard_normal(50_000)
    mask = (rng.random(50_000) > 0.3).astype(np.int64)
    assert np.array_equal(oracle.bin_values(np.zeros(npix), pix, w), b['binvalues_weighted'])
    assert np.array_equal(oracle.bin_values(np.zeros(npix), pix), b['binvalues_hits'])
    assert np.array_equal(oracle.bin_values(np.zeros(npix), pix, w, mask), b['binvalues_masked'])


def test_synthetic_inputs_reproducible(golden_dir):
    m = meta(golden_dir)
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(**m['l1_c1_config']))
    for k, v in gen['data'].items():
        assert synthetic.sha256(v) == m['l1_c1_sha256'][k], k


@pytest.fixture(scope='module')
def c1(golden_dir):
    m = meta(golden_dir)
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(**m['l1_c1_config']))
    return gen, np.load(os.path.join(golden_dir, 'golden_l1_c1.npz'))


def test_oracle_l1_matches_reference(c1):
    gen, g = c1
    out = ol1.reduce_level1(gen['data'])
    assert np.array_equal(out['averaged_tod/scan_edges'], g['averaged_tod__scan_edges'])
    # f32 nanmean sums inside the vane step are reproduced exactly
    assert relmax(out['vane/system_temperature'], g['vane__system_temperature']) == 0.0
    assert relmax(out['vane/system_gain'], g['vane__system_gain']) == 0.0
    # closed-form solves vs block_diag/spsolve and CG: rounding-level
    for k, tol in [('atmosphere/fit_values', 1e-9), ('averaged_tod/tod', 1e-8),
                   ('averaged_tod/tod_original', 1e-8), ('averaged_tod/weights', 1e-9)]:
        assert relmax(out[k], g[k.replace('/', '__')]) < tol, k
    for k in ('averaged_tod/frequency_power_spectra', 'averaged_tod/frequency_power_spectra_fits'):
        assert np.array_equal(out[k], g[k.replace('/', '__')])


@pytest.mark.parametrize('name', ['nan', 'constel', 'calib', 'tinyscan', 'f3', 'inf', 'infodd'])
def test_oracle_l1_edge_variants(golden_dir, name):
    import sys
    sys.path.insert(0, golden_dir)
    import variants
    gen = variants.make(name)
    m = meta(golden_dir)
    for k, v in gen['data'].items():
        assert synthetic.sha256(v) == m[f'l1_{name}_sha256'][k], k
    g = np.load(os.path.join(golden_dir, f'golden_l1_{name}.npz'))
    out = ol1.reduce_level1(gen['data'], source=gen['attrs']['comap']['source'])
    assert np.array_equal(out['averaged_tod/scan_edges'], g['averaged_tod__scan_edges'])
    # the calibrator branch subtracts a float32 nanmedian from the float32 cube, so
    # normalise_data's rms is a float32 nanstd in the reference: rounding ~1e-8 there
    t = 1e-7 if name == 'calib' else 1e-8
    for k, tol in [('vane/system_temperature', 0.0), ('atmosphere/fit_values', 1e-9), ('averaged_tod/tod', t),
                   ('averaged_tod/tod_original', t), ('averaged_tod/weights', t)]:
        v = out[k]
        if name == 'f3' and k.startswith('averaged_tod'):
            v = v[..., ::variants.F3_STRIDE]
        assert relmax(v, g[k.replace('/', '__')]) <= tol, k
        bad = ~np.isfinite(g[k.replace('/', '__')])         # +inf / -inf / NaN where the reference has them
        assert np.array_equal(np.asarray(v)[bad], g[k.replace('/', '__')][bad], equal_nan=True), k
    if name == 'tinyscan':
        # scans of 3 and 4 samples: the reference's fit_power_spectrum raised (dG = None)
        assert [int(e - s) for s, e in g['averaged_tod__scan_edges']][1:3] == [3, 4]
    if name == 'f3':
        assert not g['averaged_tod__tod'][2].any()          # feed 20 skipped


def test_oracle_spikes_bit_exact(golden_dir):
    import sys
    sys.path.insert(0, golden_dir)
    import variants
    from oracle import spikes
    tod, edges = variants.spikes_level2(golden_dir)
    g = np.load(os.path.join(golden_dir, 'golden_spikes.npz'))['spike_mask']
    assert np.array_equal(spikes.spike_mask(tod, edges), g)


def test_level1_averaging_oracle_vs_reference(golden_dir):
    """Level1Averaging.average_tod (generic channel binning): the NumPy restatement
    against the reference run on the C1 observation (make_golden.py --only-binning)."""
    g = np.load(os.path.join(golden_dir, 'golden_binning.npz'))
    l1 = np.load(os.path.join(golden_dir, 'golden_l1_c1.npz'))
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(**meta(golden_dir)['l1_c1_config']))
    avg, sd = ol1.level1_averaging(gen['data']['spectrometer/tod'], l1['vane__system_temperature'][0],
                                   l1['vane__system_gain'][0])
    s = int(g['stride'])
    assert np.array_equal(avg[..., ::s], g['tod'])
    assert np.array_equal(sd[..., ::s], g['tod_stddev'])
