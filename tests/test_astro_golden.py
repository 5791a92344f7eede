"""The destriper data prep's astrometric leaves against astropy 4.3.1 -- the
version the reference pins -- through golden vectors made by
tests/golden/make_astro_golden.py (the image's separate conda interpreter holds
astropy; the pipeline's Python does not).

* WCS world -> pixel (wcslib): our Calabretta & Greisen restatement
  (mapmaking/wcs.py) agrees to ~1e-12 px for CAR and ~1e-9 px for SIN / TAN, and
  COMAPData.transform_to_1d's pixel ids are identical on every point, including a
  grid placed 0.01 px from the floor(p + 0.5) edges.
* J2000 -> galactic: mapmaking/wcs.equatorial_to_galactic to 1e-5 deg of astropy's
  FK5 -> Galactic.  The reference itself rotates with healpy's
  Rotator(coord=['C','G']) (its ecliptic-based matrix, restated in astro.Rotator),
  which sits ~6e-4 deg from astropy's frame -- a property of healpy, not of the
  restatement (healpy is absent, so that matrix stays pinned only to its source).
* The Sun (get_sun, COMAPData.py:194, 218): astro.sun_radec (a Chebyshev table
  fitted to astropy 4.3.1's get_sun, tests/golden/make_sun_table.py) agrees to
  1e-8 deg, and the 10-degree Sun cut's weight mask is identical on points placed
  1e-6 .. 1e-2 deg from the cut; the almanac fallback (outside the table's
  2018-2036 range) stays within 0.01 deg.
"""
import os

import numpy as np
import pytest

from comapreduce_amd.mapmaking import astro
from comapreduce_amd.mapmaking.wcs import CelestialWCS, equatorial_to_galactic, transform_to_1d

MAPS = [
    ('car_fg9', [83.0, 12.5], [-1 / 60., 1 / 60.], [240, 240], ['RA---CAR', 'DEC--CAR'], 480, 480, 1e-10),
    ('car_ini', [10.683333, 41.268611], [-0.016666, 0.016666], [240, 240], ['RA---CAR', 'DEC--CAR'], 480, 480, 1e-10),
    ('car_gal', [30.0, 0.5], [-1 / 60., 1 / 60.], [300, 120], ['GLON-CAR', 'GLAT-CAR'], 600, 240, 1e-10),
    ('sin', [202.5, 47.2], [-1 / 60., 1 / 60.], [200, 200], ['RA---SIN', 'DEC--SIN'], 400, 400, 1e-8),
    ('tan', [150.1, 2.2], [-1 / 120., 1 / 120.], [256, 256], ['RA---TAN', 'DEC--TAN'], 512, 512, 1e-8),
]


@pytest.fixture(scope='module')
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, 'golden_astro.npz'))


def test_golden_from_reference_astropy_version(golden):
    assert str(golden['astropy_version']) == '4.3.1'


@pytest.mark.parametrize('name,crval,cdelt,crpix,ctype,nx,ny,tol', MAPS, ids=[m[0] for m in MAPS])
def test_wcs_world2pix_vs_wcslib(golden, name, crval, cdelt, crpix, ctype, nx, ny, tol):
    w = CelestialWCS(crval, cdelt, crpix, ctype)
    lon, lat = golden[f'wcs_{name}_lon'], golden[f'wcs_{name}_lat']
    rx, ry = golden[f'wcs_{name}_px'], golden[f'wcs_{name}_py']
    px, py = w.wcs_world2pix(lon, lat, 0)
    assert np.array_equal(np.isfinite(px), np.isfinite(rx))
    assert np.nanmax(np.abs(px - rx)) < tol and np.nanmax(np.abs(py - ry)) < tol
    # COMAPData.transform_to_1d on astropy's pixel coordinates
    qx, qy = np.floor(rx + 0.5), np.floor(ry + 0.5)
    qx[(qx < 0) | (qx > nx - 1)] = np.nan
    qy[(qy < 0) | (qy > ny - 1)] = np.nan
    ref = qy * nx + qx
    ref[np.isnan(ref)] = -1
    idx = transform_to_1d(lon, lat, w, nx, ny)
    assert np.array_equal(idx, ref.astype(int))
    assert (idx >= 0).sum() > 1000 and (idx < 0).sum() > 100      # on- and off-map points


def test_equatorial_to_galactic_vs_astropy(golden):
    l, b = equatorial_to_galactic(golden['gal_ra'], golden['gal_dec'])
    dl = (l - golden['gal_l'] + 180.0) % 360.0 - 180.0
    assert np.max(np.abs(dl * np.cos(np.radians(b)))) < 1e-5
    assert np.max(np.abs(b - golden['gal_b'])) < 1e-5


def test_healpy_rotator_c_to_g_vs_astropy(golden):
    ra, dec = golden['gal_ra'], golden['gal_dec']
    th, ph = astro.Rotator(coord=['C', 'G'])((90 - dec) * np.pi / 180, ra * np.pi / 180)
    l, b = np.degrees(ph) % 360.0, 90.0 - np.degrees(th)
    dl = (l - golden['gal_l'] + 180.0) % 360.0 - 180.0
    assert np.max(np.abs(dl * np.cos(np.radians(b)))) < 1e-3
    assert np.max(np.abs(b - golden['gal_b'])) < 1e-3


def _sep_deg(ra1, dec1, ra2, dec2):
    return np.degrees(astro.haversine(np.radians(dec1), np.radians(ra1), np.radians(dec2), np.radians(ra2)))


def test_sun_position_vs_astropy(golden):
    sr = np.array([astro.sun_radec(m) for m in golden['sun_mjd']])
    assert np.max(_sep_deg(sr[:, 0], sr[:, 1], golden['sun_ra'], golden['sun_dec'])) < 1e-8
    # the almanac fallback used outside the table's range
    sa = np.array([astro.sun_radec_almanac(m) for m in golden['sun_mjd']])
    assert np.max(_sep_deg(sa[:, 0], sa[:, 1], golden['sun_ra'], golden['sun_dec'])) < 0.01


def _sun_distance_with(sun_ra, sun_dec, ra, dec):
    """get_sun_centric_coords + haversine (COMAPData.py:213-236, 326-327) with a given Sun."""
    rot = astro.Rotator(rot=[sun_ra, sun_dec], inv=True)
    th, ph = rot(np.pi / 2.0 - dec * np.pi / 180.0, ra * np.pi / 180.0)
    return astro.haversine(0, 0, ph, th) * 180.0 / np.pi


def _points_near_cut(sun_ra, sun_dec, rng):
    """Equatorial points whose reference Sun 'distance' -- haversine(0, 0, phi', theta')
    of the Sun-rotated (phi', theta'), i.e. the great circle from (lat 0, lon 0) to
    (lat phi', lon theta') -- is 10 +- 1e-6 .. 1e-2 deg: placed in the rotated frame
    and rotated back with the forward Rotator."""
    delta = np.concatenate([np.logspace(-6, -2, 80), -np.logspace(-6, -2, 80)])
    rho = np.radians(10.0 + delta)
    pa = rng.uniform(0.05, np.pi - 0.05, rho.size)
    lat = np.arcsin(np.sin(rho) * np.cos(pa))                      # phi' (rotated longitude)
    lon = np.arctan2(np.sin(pa) * np.sin(rho), np.cos(rho))        # theta' (rotated colatitude) > 0
    th, ph = astro.Rotator(rot=[sun_ra, sun_dec], inv=False)(lon, lat)
    return np.degrees(ph) % 360.0, 90.0 - np.degrees(th)


def test_sun_cut_mask_identical_at_the_boundary(golden):
    """weights[ra_file < 10] = 0 (COMAPData.py:335) on points 1e-6 .. 1e-2 deg from the cut:
    our Sun gives the same mask as astropy 4.3.1's Sun through the same Rotator + haversine."""
    rng = np.random.default_rng(11)
    n_close = 0
    for k, mjd in enumerate(golden['suncut_mjd']):
        ra, dec = _points_near_cut(golden['suncut_sun_ra'][k], golden['suncut_sun_dec'][k], rng)
        want = _sun_distance_with(golden['suncut_sun_ra'][k], golden['suncut_sun_dec'][k], ra, dec)
        got, _ = astro.sun_distance_deg(ra, dec, mjd)
        assert np.max(np.abs(got - want)) < 1e-7
        assert np.array_equal(got < 10, want < 10)
        assert (want < 10).any() and (want >= 10).any()
        n_close += int(np.sum(np.abs(want - 10) < 1e-4))
        # the almanac Sun (0.007 deg off) would move some of these points across the cut
        sra, sdec = astro.sun_radec_almanac(mjd)
        alm = _sun_distance_with(sra, sdec, ra, dec)
        assert np.max(np.abs(alm - want)) > 1e-4
    assert n_close >= 200
