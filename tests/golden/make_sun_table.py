"""Chebyshev table of the Sun's apparent geocentric direction, fitted to astropy
4.3.1's ``get_sun`` -- the call the reference's destriper data prep makes
(COMAPData.py:215-218: get_sun(Time(mjd[0], format='mjd')).ra / .dec) -- and
shipped as data with the package (comapreduce_amd/mapmaking/sun_table.npz), so
``astro.sun_radec`` reproduces it without astropy / erfa (not importable by the
pipeline's Python).  Run by the image's conda interpreter, which carries astropy
4.3.1 and pyerfa:

    /opt/conda/bin/python3.9 tests/golden/make_sun_table.py

get_sun: erfa.epv00 (Earth heliocentric position, barycentric velocity; TDB from
the UTC MJD through erfa's leap-second table) + erfa.ab (stellar aberration),
returned as GCRS RA / Dec.  The table holds, per 16-day segment of UTC MJD from
2018-01-01 to 2036-01-01, degree-14 Chebyshev coefficients of the unit vector
(x, y, z) fitted at 64 Chebyshev nodes; sun_radec evaluates them and takes
atan2 / asin.  The fit residual is printed (and checked against fresh points in
tests/test_astro_golden.py); no leap second falls inside the range in astropy
4.3.1's table (the last is 2017-01-01), so UTC MJD -> TDB is smooth there.

The astropy 4.3.1 / numpy 1.26 import shims are those of make_astro_golden.py.
"""
import os

import numpy as np

for _name, _fn in (("asscalar", lambda a: a.item()), ("alen", lambda a: len(a))):
    if not hasattr(np, _name):
        setattr(np, _name, _fn)

from astropy.units.quantity_helper import function_helpers as _fh  # noqa: E402

_cat = _fh.FUNCTION_HELPERS[np.concatenate]
_fh.FUNCTION_HELPERS[np.concatenate] = lambda arrays, axis=0, out=None, dtype=None, casting='same_kind': \
    _cat(arrays, axis=axis, out=out)
from astropy.coordinates import get_sun  # noqa: E402
from astropy.time import Time  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, '..', '..', 'comapreduce_amd', 'mapmaking', 'sun_table.npz')

MJD0, MJD1 = 58119.0, 64693.0      # 2018-01-01 .. 2036-01-01 (UTC)
SEG = 16.0
DEG = 14
NODES = 64


def unit_vectors(mjd):
    s = get_sun(Time(mjd, format='mjd'))
    ra, dec = np.radians(np.asarray(s.ra.deg)), np.radians(np.asarray(s.dec.deg))
    return np.stack([np.cos(dec) * np.cos(ra), np.cos(dec) * np.sin(ra), np.sin(dec)], axis=-1)


def main():
    nseg = int(round((MJD1 - MJD0) / SEG))
    k = np.arange(NODES)
    u = np.cos(np.pi * (k + 0.5) / NODES)          # Chebyshev nodes on [-1, 1]
    mjd = (MJD0 + SEG * (np.arange(nseg)[:, None] + 0.5 * (u[None, :] + 1.0))).ravel()
    vec = unit_vectors(mjd).reshape(nseg, NODES, 3)
    coef = np.zeros((nseg, 3, DEG + 1))
    for s in range(nseg):
        for c in range(3):
            coef[s, c] = np.polynomial.chebyshev.chebfit(u, vec[s, :, c], DEG)
    # residual on points between the nodes
    rng = np.random.default_rng(5)
    test = rng.uniform(MJD0, MJD1, 4000)
    seg = np.minimum(((test - MJD0) // SEG).astype(int), nseg - 1)
    t = 2.0 * (test - (MJD0 + SEG * seg)) / SEG - 1.0
    got = np.stack([np.polynomial.chebyshev.chebval(t[i], coef[seg[i]].T) for i in range(test.size)])
    want = unit_vectors(test)
    ang = np.degrees(np.linalg.norm(got / np.linalg.norm(got, axis=1, keepdims=True) - want, axis=1))
    print(f'{nseg} segments, degree {DEG}: max residual {ang.max():.3e} deg on {test.size} fresh points')
    np.savez(OUT, mjd0=np.float64(MJD0), seg_days=np.float64(SEG), coef=coef,
             source=np.array('astropy 4.3.1 get_sun (erfa epv00 + ab), GCRS'))


if __name__ == '__main__':
    main()
