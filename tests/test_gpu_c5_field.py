"""BASELINE configs[4] as stated: 64 synthetic observations (19 feeds x 180,000 samples
each, L = 50) co-added into ONE 480 x 480 1' CAR field map, solved as one system on one
MI355X (218.9 M samples per band, 4.38 M offsets).  The reference puts every rank's
files into one map (run_destriper.py:131-189, Destriper.py:456-503); here the whole
field's operator sits in one GPU's HBM, which proves the set-up's index widths at this
size and anchors the 8-GPU strong-scaling curve (bench.py destriper_c5_field)."""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

L, NPIX, NOBS = 50, 480 * 480, 64
N_FIELD = NOBS * 19 * 180_000


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


@pytest.fixture(scope='module')
def field_band0():
    """The field's band 0: device solves (3 CG iterations at threshold 0, and converged at
    the reference's stopping rule, threshold 1e-6 / <= 100 iterations) and its inputs on
    the host."""
    import torch
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    pix, tod, w = synthetic.destriper_inputs_device(NOBS, offset_length=L, device=0, seed=5000)
    assert pix.numel() == N_FIELD
    dd = DeviceDestriper(pix, tod, w, L, NPIX, device=0)
    nnz = dd.nnz()
    res = dd.solve(threshold=0.0, niter=3)
    conv = dd.solve(threshold=1e-6, niter=100)
    out = {'x': res['x'].cpu().numpy(), 'iters': res['iters'], 'nnz': nnz,
           'maps': {k: v.cpu().numpy() for k, v in res['maps'].items()},
           'conv_x': conv['x'].cpu().numpy(), 'conv_iters': conv['iters'],
           'conv_maps': {k: v.cpu().numpy() for k, v in conv['maps'].items()},
           'p': pix.cpu().numpy(), 't': tod.cpu().numpy(), 'w': w.cpu().numpy()}
    del dd, res, conv, pix, tod, w
    torch.cuda.empty_cache()
    return out


def test_c5_field_64obs_one_band_vs_oracle(field_band0):
    """One band of the 64-observation field, 3 CG iterations, against
    oracle/destriper.py (Destriper.py:155-263, 402-453): weight / hits / naive
    bit-exact, offsets and map <= 1e-5 (north_star)."""
    import oracle.destriper as od
    f = field_band0
    assert f['iters'] == 3
    nnz_o, nnz_p = f['nnz']
    assert nnz_o == nnz_p > N_FIELD // L          # every sample on the map: each entry binned
    ref, xr, itr = od.destriper_iteration(f['p'].astype(np.int64), f['t'], f['w'], L, NPIX, threshold=0.0, niter=3)
    assert itr == 3
    for k in ('weight', 'hits', 'naive'):
        assert np.array_equal(f['maps'][k], ref[k]), k
    assert f['maps']['hits'].sum() == N_FIELD
    assert rel(f['maps']['map'], ref['map']) < 1e-5
    assert rel(f['x'], xr) < 1e-5


def test_c5_field_64obs_converged_vs_oracle(field_band0):
    """Band 0 of the 64-observation field (218.9 M samples, 4.38 M offsets) solved to the
    reference's stopping rule -- threshold 1e-6, at most 100 iterations (Destriper.py:85-152,
    402-453) -- on the device and by oracle/destriper.destriper_iteration on the host: equal
    iteration counts, weight / hits / naive bit-exact, map and offsets <= 1e-5."""
    import oracle.destriper as od
    f = field_band0
    ref, xr, itr = od.destriper_iteration(f['p'].astype(np.int64), f['t'], f['w'], L, NPIX, threshold=1e-6,
                                          niter=100)
    print(json.dumps({'field_band0_converged': {'device_iters': f['conv_iters'], 'oracle_iters': itr,
                                                'map_rel': rel(f['conv_maps']['map'], ref['map']),
                                                'x_rel': rel(f['conv_x'], xr)}}))
    assert 1 < itr < 100, itr                       # stopped by the threshold
    assert f['conv_iters'] == itr, (f['conv_iters'], itr)
    for k in ('weight', 'hits', 'naive'):
        assert np.array_equal(f['conv_maps'][k], ref[k]), k
    assert rel(f['conv_maps']['map'], ref['map']) < 1e-5
    assert rel(f['conv_x'], xr) < 1e-5


def test_c5_field_64obs_four_bands_converged(field_band0):
    """All 4 sidebands of the field as one batched system, solved to the reference's
    stopping rule (threshold 1e-6, <= 100 iterations): every band converges by the
    threshold; band 0 (the same pointing, tod and weights as the 1-band problem) has
    bit-identical weight / hits / naive maps, its first 3 iterations reproduce the 1-band
    solve and its converged solve takes the 1-band solve's iterations (which the
    converged oracle test pins) with the same map and offsets; maps finite on the hit
    pixels; band 3 equals the oracle's converged solve of its own tod and weights (iteration
    count, weight / hits / naive bit-exact, map <= 1e-5)."""
    import torch
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    pix, tod, w = synthetic.destriper_inputs_device(NOBS, offset_length=L, device=0, seed=5000, n_bands=4)
    assert tuple(tod.shape) == (4, N_FIELD)
    dd = DeviceDestriper(pix, tod, w, L, NPIX, device=0)
    t3, w3 = tod[3].cpu().numpy(), w[3].cpu().numpy()      # band 3, for the oracle below
    del pix, tod, w
    r3 = dd.solve(threshold=0.0, niter=3)
    x3 = r3['x'][0].cpu().numpy()
    m3 = r3['maps']['map'][0].cpu().numpy()
    del r3
    res = dd.solve(threshold=1e-6, niter=100)
    its = res['iters']
    x0 = res['x'][0].cpu().numpy()
    maps = {k: v.cpu().numpy() for k, v in res['maps'].items()}
    del dd, res
    torch.cuda.empty_cache()
    f = field_band0
    assert all(1 < i < 100 for i in its), its
    for k in ('weight', 'hits', 'naive'):
        assert np.array_equal(maps[k][0], f['maps'][k]), k
    assert rel(x3, f['x']) < 1e-9 and rel(m3, f['maps']['map']) < 1e-9
    assert its[0] == f['conv_iters']
    assert rel(x0, f['conv_x']) < 1e-9 and rel(maps['map'][0], f['conv_maps']['map']) < 1e-9
    for b in range(4):
        hit = maps['hits'][b] > 0
        assert maps['hits'][b].sum() == N_FIELD
        assert np.isfinite(maps['map'][b][hit]).all() and np.isfinite(maps['naive'][b][hit]).all()
    # band 3 (its own offsets and noise) against the oracle's converged solve: the batched
    # system's per-band stop test gives the reference's iteration count for that band too
    import oracle.destriper as od
    ref, xr, itr = od.destriper_iteration(f['p'].astype(np.int64), t3, w3, L, NPIX, threshold=1e-6, niter=100)
    print(json.dumps({'field_band3_converged': {'device_iters': its[3], 'oracle_iters': itr,
                                                'map_rel': rel(maps['map'][3], ref['map'])}}))
    assert its[3] == itr, (its[3], itr)
    for k in ('weight', 'hits', 'naive'):
        assert np.array_equal(maps[k][3], ref[k]), k
    assert rel(maps['map'][3], ref['map']) < 1e-5
