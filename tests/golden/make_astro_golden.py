"""Golden vectors for the destriper data prep's astrometric leaves, from astropy
4.3.1 -- the version the reference pins (requirements.txt) -- which this image
carries in a separate conda interpreter (not importable by the pipeline's Python):

    /opt/conda/bin/python3.9 tests/golden/make_astro_golden.py

* WCS world -> pixel (astropy.wcs / wcslib): the map WCS the reference's
  run_destriper.main builds (WCS(naxis=2) with crval / cdelt / crpix / ctype,
  run_destriper.py:118-122) for CAR (the COMAP fields, the parameters.ini
  Andromeda field, a GLON-CAR map), SIN and TAN, on points around each field
  including the map edges -- COMAPData.transform_to_1d calls wcs_world2pix(x, y, 0).
* The Sun: astropy.coordinates.get_sun(Time(mjd, format='mjd')).ra/.dec in degrees
  (COMAPData.py:194, 218).
* astropy's Sun at six more dates, for the 10-degree Sun-cut boundary test.
* J2000 equatorial (FK5) -> galactic by astropy, for the GLON-CAR branch
  (the reference rotates with healpy's Rotator(coord=['C','G']), COMAPData.py:411-415;
  healpy is not in the image, so this pins that rotation to astropy's frames).

Writes tests/golden/golden_astro.npz (inputs and outputs; data only).

That interpreter's numpy (1.26) no longer has np.asscalar and np.alen, which astropy 4.3.1's
units module references at import; the aliases below restore them (numpy's old
a.item() and len(a)), and its Quantity helper for np.concatenate is given the
dtype / casting keywords numpy 1.26 passes (ignored at their defaults); the
transforms themselves run in wcslib / erfa.
"""
import os

import numpy as np

for _name, _fn in (("asscalar", lambda a: a.item()), ("alen", lambda a: len(a))):
    if not hasattr(np, _name):
        setattr(np, _name, _fn)



from astropy import units as u  # noqa: E402
from astropy.units.quantity_helper import function_helpers as _fh  # noqa: E402

# numpy 1.26's np.stack passes dtype= / casting= to np.concatenate, which astropy
# 4.3.1's Quantity helper for concatenate does not accept: drop the two defaults
_cat = _fh.FUNCTION_HELPERS[np.concatenate]
_fh.FUNCTION_HELPERS[np.concatenate] = lambda arrays, axis=0, out=None, dtype=None, casting='same_kind': \
    _cat(arrays, axis=axis, out=out)
from astropy.coordinates import FK5, SkyCoord, get_sun  # noqa: E402
from astropy.time import Time  # noqa: E402
from astropy.wcs import WCS  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

# (name, crval, cdelt, crpix, ctype, nx, ny)
MAPS = [
    ('car_fg9', [83.0, 12.5], [-1 / 60., 1 / 60.], [240, 240], ['RA---CAR', 'DEC--CAR'], 480, 480),
    ('car_ini', [10.683333, 41.268611], [-0.016666, 0.016666], [240, 240], ['RA---CAR', 'DEC--CAR'], 480, 480),
    ('car_gal', [30.0, 0.5], [-1 / 60., 1 / 60.], [300, 120], ['GLON-CAR', 'GLAT-CAR'], 600, 240),
    ('sin', [202.5, 47.2], [-1 / 60., 1 / 60.], [200, 200], ['RA---SIN', 'DEC--SIN'], 400, 400),
    ('tan', [150.1, 2.2], [-1 / 120., 1 / 120.], [256, 256], ['RA---TAN', 'DEC--TAN'], 512, 512),
]


def main():
    rng = np.random.default_rng(2024)
    out = {}
    for name, crval, cdelt, crpix, ctype, nx, ny in MAPS:
        w = WCS(naxis=2)
        w.wcs.crval = crval
        w.wcs.cdelt = cdelt
        w.wcs.crpix = crpix
        w.wcs.ctype = ctype
        # points over the map and a margin around it, plus the pixel-centre grid
        # shifted by +-0.49 pixel (near, but not on, the floor(p + 0.5) edges)
        half = 0.6 * max(nx, ny) * abs(cdelt[1])
        lon = crval[0] + rng.uniform(-half, half, 4000) / np.cos(np.radians(crval[1]))
        lat = crval[1] + rng.uniform(-half, half, 4000)
        gx, gy = np.meshgrid(np.arange(0, nx, 37) + 0.49, np.arange(0, ny, 41) - 0.49)
        glon, glat = w.wcs_pix2world(gx.ravel(), gy.ravel(), 0)
        lon = np.concatenate([lon, glon])
        lat = np.concatenate([lat, glat])
        px, py = w.wcs_world2pix(lon, lat, 0)
        out[f'wcs_{name}_lon'] = lon
        out[f'wcs_{name}_lat'] = lat
        out[f'wcs_{name}_px'] = px
        out[f'wcs_{name}_py'] = py
    mjd = 59000.0 + np.concatenate([np.arange(0, 1100, 37.3), [0.25, 100.75, 365.5]])
    sun = get_sun(Time(mjd, format='mjd'))
    out['sun_mjd'] = mjd
    out['sun_ra'] = np.asarray(sun.ra.deg)
    out['sun_dec'] = np.asarray(sun.dec.deg)
    # the Sun at six dates for the 10-degree Sun-cut boundary test (COMAPData.py:326-335;
    # tests/test_astro_golden.py places points 1e-6 .. 1e-2 deg from the cut around it)
    cut_mjd = 58300.0 + np.array([0.0, 211.37, 512.9, 1300.25, 2111.6, 3650.01])
    csun = get_sun(Time(cut_mjd, format='mjd'))
    out['suncut_mjd'] = cut_mjd
    out['suncut_sun_ra'] = np.asarray(csun.ra.deg)
    out['suncut_sun_dec'] = np.asarray(csun.dec.deg)
    ra = rng.uniform(0, 360, 2000)
    dec = np.degrees(np.arcsin(rng.uniform(-1, 1, 2000)))
    g = SkyCoord(ra=ra * u.deg, dec=dec * u.deg, frame=FK5(equinox='J2000')).galactic
    out['gal_ra'] = ra
    out['gal_dec'] = dec
    out['gal_l'] = np.asarray(g.l.deg)
    out['gal_b'] = np.asarray(g.b.deg)
    import astropy
    out['astropy_version'] = np.array(astropy.__version__)
    np.savez_compressed(os.path.join(HERE, 'golden_astro.npz'), **out)
    print('wrote golden_astro.npz with astropy', astropy.__version__)


if __name__ == '__main__':
    main()
