"""The batched host vane search (gpu.find_hot_cold_batch) against the
per-series restatement of VaneCalibration.py:86-141 (find_hot_cold_from_tod,
itself pinned to the reference through the vane goldens): identical hot and
cold sample offsets on vane-like windows, noise, NaNs, flat rows and odd
lengths."""
import numpy as np
import pytest

from comapreduce_amd.gpu import find_hot_cold_batch, find_hot_cold_from_tod
from comapreduce_amd import synthetic


def per_series(ba):
    hot, cold, hoff, coff = [], [], [0], [0]
    for row in ba:
        h, c = find_hot_cold_from_tod(row)
        if h is None or c is None:
            h = c = np.zeros(0, dtype=int)
        hot.append(h)
        cold.append(c)
        hoff.append(hoff[-1] + len(h))
        coff.append(coff[-1] + len(c))
    return np.concatenate(hot), np.array(hoff), np.concatenate(cold), np.array(coff)


def check(ba):
    h, ho, c, co = find_hot_cold_batch(ba)
    rh, rho, rc, rco = per_series(ba)
    assert np.array_equal(ho, rho) and np.array_equal(co, rco)
    assert np.array_equal(h, rh) and np.array_equal(c, rc)


def vane_window(rng, n, L, hot=(100, 500), noise=0.01, step=3.0):
    x = 1.0 + noise * rng.standard_normal((n, L))
    ramp = np.clip((np.arange(L) - hot[0]) / 20.0, 0, 1) * np.clip((hot[1] - np.arange(L)) / 20.0, 0, 1)
    x += step * ramp
    return x.astype(np.float32)


@pytest.mark.parametrize('seed', range(6))
def test_vane_like(seed):
    rng = np.random.default_rng(seed)
    L = [1000, 999, 1001, 400, 2000, 37][seed]
    check(vane_window(rng, 76, L, hot=(L // 10, L // 2), noise=[1e-2, 1e-3, 1e-4, 5e-2, 1e-2, 1e-3][seed]))


def test_noise_nan_flat():
    rng = np.random.default_rng(11)
    ba = vane_window(rng, 40, 800)
    ba[3, 10:20] = np.nan
    ba[4, :] = 2.0                    # flat row: rng = 0 -> NaN comparisons, no samples
    ba[5] = rng.standard_normal(800).astype(np.float32)
    ba[6, 300] = np.nan
    ba[7, :] = np.nan
    ba[8] *= -1                       # inverted: hot search sees the dip
    with np.errstate(all='ignore'):
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            check(ba)


def test_synthetic_vane_windows():
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(n_feeds=2, n_samples=4000, obs_id=5))
    ba = np.asarray(gen['data']['spectrometer/band_average'])
    feats = synthetic_features(gen)
    idx = np.nonzero(np.diff(feats == 13))[0] + 1
    s, e = idx[0], idx[1]
    check(np.ascontiguousarray(ba[:, :, s:e].reshape(-1, e - s)))


def synthetic_features(gen):
    f = np.asarray(gen['data']['spectrometer/features'])
    out = np.zeros(f.shape, dtype=int)
    nz = f != 0
    out[nz] = np.floor(np.log(f[nz]) / np.log(2)).astype(int)
    return out
