"""GPU parity of the L1 -> L2 path against the reference golden vectors and
the CPU oracle (tolerances from BASELINE.json north_star: bit-exact for
indices / median selections, <= 1e-5 relative for calibrated TOD, spectra)."""
import json
import os

import numpy as np
import pytest

import oracle
from comapreduce_amd import synthetic
from comapreduce_amd.pipeline.datahandling import COMAPLevel2, level1_from_dict

pytestmark = pytest.mark.gpu
RTOL = 1e-5   # north_star: "within 1e-5 relative"


def relmax(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin), 'NaN pattern differs'
    return np.max(np.abs(a[fin] - b[fin])) / max(np.max(np.abs(b[fin])), 1e-300)


@pytest.fixture(scope='module')
def meta(golden_dir):
    return json.load(open(os.path.join(golden_dir, 'golden_meta.json')))


@pytest.fixture(scope='module')
def c1_run(meta, golden_dir):
    from comapreduce_amd import Analysis as A
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(**meta['l1_c1_config']))
    data = level1_from_dict(gen)
    level2 = COMAPLevel2(filename='/nonexistent/none.hd5')
    for cls in (A.MeasureSystemTemperature, A.AtmosphereRemoval, A.Level1AveragingGainCorrection):
        st = cls(level2=level2)
        assert st(data, level2)
        level2.update(st)
    return gen, data, level2, np.load(os.path.join(golden_dir, 'golden_l1_c1.npz'))


def test_medfilt_dropin_bit_exact(meta, golden_dir):
    from comapreduce_amd.tools.medfilt import medfilt
    g = np.load(os.path.join(golden_dir, 'golden_medfilt.npz'))
    for seed, n, w in meta['medfilt_cases']:
        x = np.random.default_rng(seed).standard_normal(n)
        y = medfilt(x, w)
        assert y is x
        assert np.array_equal(x, g[f'medfilt_{seed}_{n}_{w}']), (seed, n, w)


def _median_path(path, monkeypatch):
    """'sort': segments sorted in LDS (longer ones on the device-wide sort) + the
    wavelet-matrix walk (the default); 'devsort': every segment on the device-wide
    segmented sort; 'bitmap': the chunked bitmap walk (windows > 16384)."""
    monkeypatch.setenv('COMAP_MEDIAN_BLOCKSORT', '0' if path == 'devsort' else '1')
    monkeypatch.setenv('COMAP_MEDIAN_WALK', 'bitmap' if path == 'bitmap' else 'wm')


@pytest.mark.parametrize('path', ['sort', 'devsort', 'bitmap'])
def test_medfilt_dropin_ties_and_edges(path, monkeypatch):
    """Every device median path: either sort of the segments, either walk."""
    _median_path(path, monkeypatch)
    from comapreduce_amd.tools.medfilt import medfilt
    rng = np.random.default_rng(9)
    for n, w in [(6000, 6000), (12000, 6000), (7681, 7681), (513, 400), (2048, 2), (100, 1), (3000, 5),
                 (20000, 9001), (16129, 16129), (700, 256), (1000, 255)]:
        x = np.round(rng.standard_normal(n), 1)   # heavy ties
        assert np.array_equal(medfilt(x.copy(), w), oracle.medfilt(x.copy(), w)), (n, w)


def _inf_series(rng, n):
    """Rounded normals (ties) with scattered +-inf, a run of +inf that makes window
    medians +inf and a following run of -inf whose windows' middle pair is -inf / +inf
    (the even-w mean is NaN, as Mediator::getMedian's (a + b) / 2 gives)."""
    x = np.round(rng.standard_normal(n), 1)
    x[rng.random(n) < 0.03] = np.inf
    x[rng.random(n) < 0.03] = -np.inf
    a = n // 3
    x[a:a + 300] = np.inf
    x[a + 300:a + 600] = -np.inf
    return x


@pytest.mark.parametrize('path', ['sort', 'devsort', 'bitmap'])
def test_medfilt_dropin_infinities(path, monkeypatch):
    """+-inf input (the reference's two-heap orders +-inf like any value, so every
    window median is an order statistic): drop-in medfilt and the reflect-padded batch ==
    oracle.medfilt, which test_oracle_golden pins to the reference's compiled filter on
    this input."""
    _median_path(path, monkeypatch)
    from comapreduce_amd.tools.medfilt import medfilt, medfilt_batch
    rng = np.random.default_rng(31)
    for n, w in [(5000, 400), (4000, 401), (3000, 6), (9000, 6000)]:
        x = _inf_series(rng, n)
        assert np.array_equal(medfilt(x.copy(), w), oracle.medfilt(x.copy(), w), equal_nan=True), (n, w)
    series = [_inf_series(rng, n) for n in (1201, 5000, 900)]
    for s, g in zip(series, medfilt_batch(series, 400, reflect=True)):
        z = np.concatenate((s[::-1], s, s[::-1]))
        assert np.array_equal(g, oracle.medfilt(z, 400)[s.size:2 * s.size], equal_nan=True), s.size


def test_medfilt_dropin_nan_fixtures(golden_dir):
    """NaN input through the drop-in (comap_medfilt_f64) and the batched reflect-padded
    form (comap_medfilt_batch_f64): the two-heap replay == the reference's compiled filter
    on the committed known-answer fixtures, bit for bit, NaN positions included
    (tests/golden/make_medfilt_nan.py)."""
    from comapreduce_amd.tools.medfilt import medfilt, medfilt_batch
    g = np.load(os.path.join(golden_dir, 'golden_medfilt_nan.npz'))
    names = sorted(k[2:] for k in g.files if k.startswith('x_'))
    assert len(names) == 12
    for name in names:
        x, y, w, r = g[f'x_{name}'], g[f'y_{name}'], int(g[f'w_{name}']), bool(g[f'r_{name}'])
        if r:
            got = medfilt_batch([x], w, reflect=True)[0]
        else:
            got = medfilt(x.copy(), w)
        assert np.array_equal(got, y, equal_nan=True), name
    # a batch mixing NaN-bearing series (replayed) with NaN-free ones (order statistics)
    plain = [np.round(np.random.default_rng(s).standard_normal(n), 1) for s, n in ((1, 2000), (2, 4000))]
    series = [plain[0], g['x_single_w400'], plain[1], g['x_head_tail_w100']]
    for s, got in zip(series, medfilt_batch(series, 400)):
        assert np.array_equal(got, oracle.medfilt(s.copy(), 400), equal_nan=True)


@pytest.mark.parametrize('path', ['sort', 'devsort', 'bitmap'])
def test_medfilt_long_series_split(path, monkeypatch):
    """Series longer than one median sub-job / segment are split internally."""
    _median_path(path, monkeypatch)
    from comapreduce_amd.tools.medfilt import medfilt, medfilt_batch
    rng = np.random.default_rng(10)
    x = np.round(rng.standard_normal(150_001), 2)
    assert np.array_equal(medfilt(x.copy(), 401), oracle.medfilt(x.copy(), 401))
    y = np.round(rng.standard_normal(140_000), 2)
    got = medfilt_batch([y], 400, reflect=True)[0]
    z = np.concatenate((y[::-1], y, y[::-1]))
    assert np.array_equal(got, oracle.medfilt(z, 400)[y.size:2 * y.size])


@pytest.mark.parametrize('key32,lc,S', [('1', 'wm', ''), ('0', 'wm', ''), ('1', 'wm', '7'), ('1', '128', ''),
                                        ('0', '128', ''), ('1', '64', ''), ('1', '256', ''),
                                        ('1', '512', ''), ('1', '128', '1'), ('1', '128', '3'), ('1', '64', '16')])
def test_medfilt_sort_proxy_runs(key32, lc, S, monkeypatch):
    """Global-sort path with 32-bit proxy keys: values that round to the same
    f32 but differ in f64 (short runs: fixed in place; runs > 32: the segment is
    re-sorted on u64 keys), signed zeros and negative values; u64-key path; the
    wavelet-matrix walk (one or several segments per series), and the bitmap walk with
    64/256/512-output chunks and 1..16 chunks per walk workgroup for comparison."""
    monkeypatch.setenv('COMAP_MEDIAN_KEY32', key32)
    if lc == 'wm':
        monkeypatch.setenv('COMAP_MEDIAN_WALK', lc)
        if S:
            monkeypatch.setenv('COMAP_MEDIAN_WMSEGS', S)   # segments to fill the chip (splits every series)
        lc, S = '128', ''
    else:
        monkeypatch.setenv('COMAP_MEDIAN_WALK', 'bitmap')
    monkeypatch.setenv('COMAP_MEDIAN_L', lc)
    if S:
        monkeypatch.setenv('COMAP_MEDIAN_S', S)      # chunks per walk workgroup (bitmaps slid between them)
    from comapreduce_amd.tools.medfilt import medfilt, medfilt_batch
    rng = np.random.default_rng(12)
    n = 20000
    eps = rng.integers(0, 5, n) * 1e-13
    short = np.round(rng.standard_normal(n), 4) + eps            # runs of ~1-3 equal proxies
    long_ = np.round(rng.standard_normal(n), 1) + eps            # runs of hundreds -> segment re-sort
    flat = 1.0 + rng.integers(0, 40, n) * 2.0 ** -45              # one proxy for the whole series
    zeros = np.where(rng.random(n) < 0.5, 0.0, -0.0) * (rng.random(n) < 0.9) + (rng.random(n) < 0.1) * -1e-300
    cluster = rng.standard_normal(n) * 1e6                          # wide range: coarse proxy buckets ...
    cluster[rng.choice(n, 300, replace=False)] = 1.0 + np.arange(300) * 1e-12   # ... one holds a 300-run
    for x, w in ((short, 6000), (long_, 6000), (flat, 401), (zeros, 400), (short[:7000], 7000), (cluster, 6000)):
        assert np.array_equal(medfilt(x.copy(), w), oracle.medfilt(x.copy(), w)), (w, x[:3])
    series = [short, long_[:9000], flat[:6500]]
    got = medfilt_batch(series, 6000, reflect=True)
    for s, g in zip(series, got):
        z = np.concatenate((s[::-1], s, s[::-1]))
        assert np.array_equal(g, oracle.medfilt(z, 6000)[s.size:2 * s.size])


def test_binvalues_dropin_bit_exact(golden_dir):
    from comapreduce_amd.tools.binfuncs import binValues
    b = np.load(os.path.join(golden_dir, 'golden_binvalues.npz'))
    rng = np.random.default_rng(21)
    npix = 1000
    pix = rng.integers(-50, npix + 50, 50_000).astype(np.int64)
    w = rng.standard_normal(50_000)
    mask = (rng.random(50_000) > 0.3).astype(np.int64)
    for args, key in [((w,), 'binvalues_weighted'), ((), 'binvalues_hits'), ((w, mask), 'binvalues_masked')]:
        img = np.zeros(npix)
        binValues(img, pix, *args)
        assert np.array_equal(img, b[key]), key


def test_l1_vane_vs_reference(c1_run):
    """Bit-exact: the kernel reproduces numpy's float32 pairwise nanmean."""
    _, _, l2, g = c1_run
    assert np.array_equal(l2['vane/system_temperature'], g['vane__system_temperature'])
    assert np.array_equal(l2['vane/system_gain'], g['vane__system_gain'])


def test_l1_atmosphere_vs_reference(c1_run):
    _, _, l2, g = c1_run
    assert relmax(l2['atmosphere/fit_values'], g['atmosphere__fit_values']) < RTOL


def test_l1_averaged_tod_vs_reference(c1_run):
    _, _, l2, g = c1_run
    assert np.array_equal(l2['averaged_tod/scan_edges'], g['averaged_tod__scan_edges'])
    for k in ('tod', 'tod_original', 'weights'):
        assert relmax(l2[f'averaged_tod/{k}'], g[f'averaged_tod__{k}']) < RTOL, k
    for k in ('frequency_power_spectra', 'frequency_power_spectra_fits'):
        assert np.array_equal(l2[f'averaged_tod/{k}'], g[f'averaged_tod__{k}'])


def test_l1_median_selection_bit_exact(c1_run):
    """The device median of the device band mean == the oracle medfilt on the
    same (reflect-padded) input vector, bit for bit."""
    _, data, _, _ = c1_run
    obs = data._gpu_observation
    mb = obs.debug(4)
    mf = obs.debug(1)
    for f, s, t0, n in obs.units:
        if n < 12000:
            continue
        for b in range(4):
            m = mb[f, b, t0:t0 + n]
            pad = np.concatenate([m[::-1], m, m[::-1]])
            ref = oracle.medfilt(pad, 6000)[n:2 * n]
            assert np.array_equal(mf[f, b, t0:t0 + n], ref), (f, s, b)


@pytest.mark.parametrize('name', ['nan', 'constel', 'calib', 'tinyscan', 'f3', 'inf', 'infodd'])
def test_l1_edge_variants_vs_reference(golden_dir, name):
    """NaN fill/select_time, constant-elevation, calibrator and +-inf paths on the device."""
    import sys
    sys.path.insert(0, golden_dir)
    import variants
    from comapreduce_amd import Analysis as A
    gen = variants.make(name)
    data = level1_from_dict(gen)
    level2 = COMAPLevel2(filename='/nonexistent/none.hd5')
    for cls in (A.MeasureSystemTemperature, A.AtmosphereRemoval, A.Level1AveragingGainCorrection):
        st = cls(level2=level2)
        assert st(data, level2)
        level2.update(st)
    g = np.load(os.path.join(golden_dir, f'golden_l1_{name}.npz'))
    assert np.array_equal(level2['averaged_tod/scan_edges'], g['averaged_tod__scan_edges'])
    for k in ('vane/system_temperature', 'vane/system_gain'):
        assert np.array_equal(level2[k], g[k.replace('/', '__')]), (name, k)
    for k in ('atmosphere/fit_values', 'averaged_tod/tod', 'averaged_tod/tod_original', 'averaged_tod/weights'):
        v = np.asarray(level2[k])
        if name == 'f3' and k.startswith('averaged_tod'):
            v = v[..., ::variants.F3_STRIDE]
        assert relmax(v, g[k.replace('/', '__')]) < RTOL, (name, k)
        bad = ~np.isfinite(g[k.replace('/', '__')])         # +inf / -inf / NaN as the reference has them
        assert np.array_equal(v[bad], g[k.replace('/', '__')][bad], equal_nan=True), (name, k)


def test_spikes_stage_bit_exact(golden_dir):
    import sys
    sys.path.insert(0, golden_dir)
    import variants
    from comapreduce_amd import Analysis as A
    tod, edges = variants.spikes_level2(golden_dir)
    l2 = COMAPLevel2(filename='/nonexistent/spk.hd5')
    l2['averaged_tod/tod'] = tod
    l2['averaged_tod/scan_edges'] = edges
    l2.set_attrs('comap', 'source', 'Field00')
    st = A.Spikes(level2=l2)
    assert st(l2, l2)
    g = np.load(os.path.join(golden_dir, 'golden_spikes.npz'))['spike_mask']
    assert np.array_equal(st.data['spikes/spike_mask'], g)


def test_level1_averaging_vs_reference(meta, golden_dir):
    """Level1Averaging (Level1Averaging.py:249-321), called as the reference's
    one-argument __call__, against the reference golden (C1 observation)."""
    from comapreduce_amd import Analysis as A
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(**meta['l1_c1_config']))
    data = level1_from_dict(gen)
    level2 = COMAPLevel2(filename='/nonexistent/none.hd5')
    vane = A.MeasureSystemTemperature(level2=level2)
    assert vane(data, level2)
    level2.update(vane)
    st = A.Level1Averaging(level2=level2)
    assert st(data)
    g = np.load(os.path.join(golden_dir, 'golden_binning.npz'))
    s = int(g['stride'])
    assert st.tod.shape == (1, 4, 2, meta['l1_c1_config']['n_samples'])
    assert relmax(st.tod[..., ::s], g['tod']) < 1e-12
    assert relmax(st.tod_stddev[..., ::s], g['tod_stddev']) < 1e-9
    # half-size bins exercise the generic bin loop
    st4 = A.Level1Averaging(level2=level2, frequency_bin_size=256)
    assert st4(data, level2)
    ref_a, ref_s = __import__('oracle.l1', fromlist=['x']).level1_averaging(
        gen['data']['spectrometer/tod'], np.asarray(level2['vane/system_temperature'])[0],
        np.asarray(level2['vane/system_gain'])[0], 256)
    assert relmax(st4.tod, ref_a) < 1e-12
    assert relmax(st4.tod_stddev, ref_s) < 1e-9


# ---------------------------------------------------------------- multi-feed observation + C3 shards
F3 = dict(n_feeds=3, n_samples=30_000, obs_id=5, feed_numbers=(1, 2, 20))


@pytest.fixture(scope='module')
def f3_gen():
    return synthetic.generate_level1(synthetic.SyntheticConfig(**F3))


def _reduce(data):
    from comapreduce_amd import Analysis as A
    level2 = COMAPLevel2(filename='/nonexistent/none.hd5')
    for cls in (A.MeasureSystemTemperature, A.AtmosphereRemoval, A.Level1AveragingGainCorrection):
        st = cls(level2=level2)
        assert st(data, level2)
        level2.update(st)
    return level2


KEYS = ('vane/system_temperature', 'vane/system_gain', 'atmosphere/fit_values', 'averaged_tod/tod',
        'averaged_tod/tod_original', 'averaged_tod/weights')


def test_multi_feed_observation_vs_oracle(f3_gen):
    """F = 3 feeds, every (feed, scan) unit, against oracle.l1.reduce_level1; feed
    number 20 is skipped by the reducer (Level1Averaging.py:817-818): its
    averaged_tod rows stay 0 while its vane and atmosphere are still computed."""
    import oracle.l1 as ol1
    l2 = _reduce(level1_from_dict(f3_gen))
    ref = ol1.reduce_level1(f3_gen['data'])
    for k in ('vane/system_temperature', 'vane/system_gain'):
        assert np.array_equal(l2[k], ref[k]), k
    for k in KEYS[2:]:
        assert relmax(l2[k], ref[k]) < RTOL, k
    for k in ('averaged_tod/tod', 'averaged_tod/tod_original', 'averaged_tod/weights'):
        assert not np.asarray(l2[k])[2].any(), k
        assert np.asarray(l2[k])[:2].any(), k
    assert np.isfinite(np.asarray(l2['atmosphere/fit_values'])[:, 2, :, :, 10:1014][..., :500]).all()


@pytest.mark.parametrize('world', [2, 3])
def test_shards_bit_identical(f3_gen, world):
    """C3 on the device: each shard (its feeds, its units only) reduced by its own
    plan; the assembled owned slices equal the unsharded device run bit for bit."""
    from comapreduce_amd.pipeline import sharding
    full = _reduce(level1_from_dict(f3_gen))
    shards, outs = [], []
    for r in range(world):
        sh, part = sharding.shard_level1(level1_from_dict(f3_gen), r, world)
        l2 = _reduce(part)
        shards.append(sh)
        outs.append({k: l2[k] for k in KEYS})
    S = len(full['averaged_tod/scan_edges'])
    got = sharding.assemble(shards, outs, 3, S, F3['n_samples'])
    for k in KEYS:
        assert np.array_equal(got[k], np.asarray(full[k]), equal_nan=True), k


def test_context_keeps_current_device():
    """Creating a context and running a drop-in leave torch's current device alone."""
    import torch
    from comapreduce_amd import _native as N
    from comapreduce_amd.tools.medfilt import medfilt_batch
    before = torch.cuda.current_device()
    for d in range(torch.cuda.device_count()):
        N.ctx(d)
        assert torch.cuda.current_device() == before
    medfilt_batch([np.arange(1000.0)], 401, reflect=True)
    assert torch.cuda.current_device() == before


def test_nan_fill_leaves_raw_cube(golden_dir):
    """fill_bad_data is applied for the L1AGC reduction only: afterwards the resident
    cube holds its NaNs again, so a later stage (Level1Averaging, a re-run of
    L1AGC) sees the raw data, as every reference stage does (DataHandling.py:176-177)."""
    import sys
    import oracle.l1 as ol1
    sys.path.insert(0, golden_dir)
    import variants
    from comapreduce_amd import Analysis as A
    gen = variants.make('nan')
    raw = gen['data']['spectrometer/tod'].copy()
    data = level1_from_dict(gen)
    l2 = _reduce(data)
    dev = data._gpu_observation.tod.cpu().numpy()
    assert np.array_equal(np.isnan(dev), np.isnan(raw))
    assert np.array_equal(dev, raw, equal_nan=True)
    st = A.Level1Averaging(level2=l2)
    assert st(data, l2)
    ref_a, ref_s = ol1.level1_averaging(raw, np.asarray(l2['vane/system_temperature'])[0],
                                        np.asarray(l2['vane/system_gain'])[0], 512)
    assert relmax(st.tod, ref_a) < 1e-12
    # a second L1AGC on the same plan gives the same outputs as the first
    again = A.Level1AveragingGainCorrection(level2=l2)
    assert again(data, l2)
    assert np.array_equal(again.tod_cleaned, np.asarray(l2['averaged_tod/tod']), equal_nan=True)


def test_scan_alignment_residues_vs_oracle():
    """Pass A (k_moments) forms normalise_data's scan-relative stride-4 difference
    pairs from unaligned scan starts: scans starting at every residue mod 4, with
    every length residue and one short scan (no median band), against
    oracle.l1.reduce_level1 (Level1Averaging.py:642-679)."""
    import oracle.l1 as ol1
    T = 59_000
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(n_feeds=1, n_samples=T, obs_id=21))
    st = np.zeros(T, dtype=np.int64)
    for a, b in ((1500, 15502), (16502, 29500), (30500, 43503), (44503, 57503), (58200, 58707)):
        st[a:b] = 1
    gen['data']['hk/antenna0/deTracker/lissajous_status'] = st
    edges = synthetic.scan_edges_from_status(st)
    assert sorted({int(s) % 4 for s, _ in edges}) == [0, 1, 2, 3]
    assert sorted({int(e - s) % 4 for s, e in edges}) == [0, 1, 2, 3]
    l2 = _reduce(level1_from_dict(gen))
    ref = ol1.reduce_level1(gen['data'])
    assert np.asarray(l2['averaged_tod/scan_edges']).tolist() == np.asarray(ref['averaged_tod/scan_edges']).tolist()
    for k in KEYS[2:]:
        assert relmax(l2[k], ref[k]) < RTOL, k
