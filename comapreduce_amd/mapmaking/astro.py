"""Sky rotations and the Sun's position for the destriper data prep.

The reference calls ``healpy.rotator.Rotator`` (COMAPData.py:199, 223, 412)
and ``astropy.coordinates.get_sun`` (COMAPData.py:194, 218); neither package
is in this image.  ``Rotator`` below restates healpy's matrix construction
(``euler_matrix_new`` with the default 'ZYX' Euler type, ``rot=[lon, lat,
psi]`` in degrees, ``get_rotation_matrix`` negating the latitude angle,
``get_coordconv_matrix`` for 'C'->'G', ``inv`` transposing) and its
``__call__(theta, phi)`` (ang2vec -> matrix -> vec2ang with phi in
(-pi, pi]).  ``sun_radec`` evaluates a Chebyshev table of the Sun's
apparent geocentric direction fitted to astropy 4.3.1's ``get_sun`` (erfa
epv00 + aberration, GCRS; the reference's pinned version) by
tests/golden/make_sun_table.py and shipped as data (``sun_table.npz``, UTC MJD
2018-01-01 .. 2036-01-01, fit residual 1.5e-10 deg); outside that range it falls
back to the Astronomical Almanac low-precision ephemeris (~0.007 deg from
get_sun), which only moves samples within that distance of the reference's
10-degree Sun cut.  healpy is absent, so the Rotator is pinned to healpy's source
only; the golden harness uses these same functions as its stand-ins, so
everything downstream of them is pinned.
"""
from __future__ import annotations

import os

import numpy as np

_SUN_TABLE = None


def euler_matrix_zyx(a1, a2, a3):
    c1, s1 = np.cos(a1), np.sin(a1)
    c2, s2 = np.cos(a2), np.sin(a2)
    c3, s3 = np.cos(a3), np.sin(a3)
    m1 = np.array([[c1, -s1, 0.0], [s1, c1, 0.0], [0.0, 0.0, 1.0]])
    m2 = np.array([[c2, 0.0, s2], [0.0, 1.0, 0.0], [-s2, 0.0, c2]])
    m3 = np.array([[1.0, 0.0, 0.0], [0.0, c3, -s3], [0.0, s3, c3]])
    return np.dot(m3.T, np.dot(m2.T, m1.T))


def coordconv_matrix(coord):
    if coord is None or coord[0] == coord[1]:
        return np.identity(3)
    eps = (23.452294 - 0.0130125 - 1.63889e-6 + 5.02778e-7) * np.pi / 180.0
    e2g = np.array([[-0.054882486, -0.993821033, -0.096476249],
                    [0.494116468, -0.110993846, 0.862281440],
                    [-0.867661702, -0.000346354, 0.497154957]])
    e2q = np.array([[1.0, 0.0, 0.0], [0.0, np.cos(eps), -np.sin(eps)], [0.0, np.sin(eps), np.cos(eps)]])
    q2e = np.linalg.inv(e2q)
    g2e = np.linalg.inv(e2g)
    table = {('E', 'G'): e2g, ('G', 'E'): g2e, ('E', 'C'): e2q, ('C', 'E'): q2e,
             ('C', 'G'): np.dot(e2g, q2e), ('G', 'C'): np.dot(e2q, g2e)}
    return table[(coord[0].upper(), coord[1].upper())]


class Rotator:
    """healpy.rotator.Rotator for a single (rot, coord, inv) triple."""

    def __init__(self, rot=None, coord=None, inv=False, deg=True):
        r = np.zeros(3)
        if rot is not None:
            v = np.asarray(rot, dtype=np.float64).ravel() * (np.pi / 180.0 if deg else 1.0)
            r[:v.size] = v
        rn = euler_matrix_zyx(r[0], -r[1], r[2])
        xn = np.dot(rn, coordconv_matrix(coord))
        self.mat = xn.T if inv else xn

    def __call__(self, theta, phi):
        theta = np.asarray(theta, dtype=np.float64)
        phi = np.asarray(phi, dtype=np.float64)
        st = np.sin(theta)
        v = np.array([st * np.cos(phi), st * np.sin(phi), np.cos(theta)])
        x, y, z = np.tensordot(self.mat, v, axes=(1, 0))
        r = np.sqrt(x * x + y * y + z * z)
        return np.array([np.arccos(z / r), np.arctan2(y, x)])


def _sun_table():
    global _SUN_TABLE
    if _SUN_TABLE is None:
        with np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'sun_table.npz')) as z:
            _SUN_TABLE = (float(z['mjd0']), float(z['seg_days']), np.array(z['coef']))
    return _SUN_TABLE


def sun_radec_almanac(mjd):
    """Apparent solar RA/Dec (deg) referred to the J2000 equinox: the Astronomical
    Almanac's low-precision formulae (~0.01 deg, 1950-2050)."""
    n = float(mjd) + 2400000.5 - 2451545.0
    L = 280.460 + 0.9856474 * n
    g = np.deg2rad(357.528 + 0.9856003 * n)
    lam = L + 1.915 * np.sin(g) + 0.020 * np.sin(2 * g)
    lam -= 1.396971 * (n / 36525.0)           # precess ecliptic longitude back to J2000
    eps = np.deg2rad(23.4392911)
    lr = np.deg2rad(lam)
    ra = np.rad2deg(np.arctan2(np.cos(eps) * np.sin(lr), np.cos(lr))) % 360.0
    dec = np.rad2deg(np.arcsin(np.sin(eps) * np.sin(lr)))
    return ra, dec


def sun_radec(mjd):
    """get_sun(Time(mjd, format='mjd')).ra.deg / .dec.deg (COMAPData.py:215-218):
    the Chebyshev table of astropy 4.3.1's get_sun inside its range (UTC MJD), the
    almanac outside it."""
    mjd0, seg, coef = _sun_table()
    k = int(np.floor((float(mjd) - mjd0) / seg))
    if not 0 <= k < coef.shape[0]:
        return sun_radec_almanac(mjd)
    t = 2.0 * (float(mjd) - (mjd0 + seg * k)) / seg - 1.0
    x, y, z = np.polynomial.chebyshev.chebval(t, coef[k].T)
    ra = np.rad2deg(np.arctan2(y, x)) % 360.0
    dec = np.rad2deg(np.arcsin(z / np.sqrt(x * x + y * y + z * z)))
    return ra, dec


def haversine(theta1, phi1, theta2, phi2):
    """COMAPData.haversine (COMAPData.py:235-236)."""
    return 2 * np.arcsin(np.sqrt(np.sin((theta2 - theta1) / 2) ** 2
                                 + np.cos(theta1) * np.cos(theta2) * np.sin((phi2 - phi1) / 2) ** 2))


def sun_distance_deg(ra, dec, mjd0):
    """get_sun_centric_coords + haversine as used by get_tod
    (COMAPData.py:213-232, 326-327): returns (ra_file, dec_file) exactly as
    the reference stores them -- the haversine of the rotated (phi, theta)
    pair in degrees, and the rotated colatitude in radians."""
    sra, sdec = sun_radec(mjd0)
    rot = Rotator(rot=[sra, sdec], inv=True)
    theta = np.pi / 2.0 - np.asarray(dec, dtype=np.float64) * np.pi / 180.0
    phi = np.asarray(ra, dtype=np.float64) * np.pi / 180.0
    good = np.isfinite(ra) & np.isfinite(dec)
    theta = theta.copy()
    phi = phi.copy()
    t, p = rot(theta[good], phi[good])
    theta[good], phi[good] = t, p
    return haversine(0, 0, phi, theta) * 180.0 / np.pi, theta
