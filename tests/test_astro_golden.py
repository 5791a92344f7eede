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
* The Sun (get_sun, COMAPData.py:194, 218): astro.sun_radec (low-precision
  almanac) is within 0.01 deg of astropy's GCRS Sun; only samples that close to
  the 10-degree Sun cut could change side.
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


def test_sun_position_vs_astropy(golden):
    sr = np.array([astro.sun_radec(m) for m in golden['sun_mjd']])
    dra = (sr[:, 0] - golden['sun_ra'] + 180.0) % 360.0 - 180.0
    assert np.max(np.abs(dra * np.cos(np.radians(golden['sun_dec'])))) < 0.01
    assert np.max(np.abs(sr[:, 1] - golden['sun_dec'])) < 0.01
