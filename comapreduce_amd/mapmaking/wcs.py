"""Minimal FITS celestial WCS (world -> pixel) for the destriper's map grid.

The reference builds an ``astropy.wcs.WCS`` (run_destriper.py:118-128) and
calls ``wcs_world2pix(x, y, 0)`` (COMAPData.py:98).  astropy/wcslib are not
in this image, so this restates the Calabretta & Greisen (2002) pipeline for
the projections the COMAP configs use -- CAR (cylindrical, (phi0, theta0) =
(0, 0)), SIN and TAN (zenithal, (0, 90)) -- with CDELT scaling and default
LONPOLE/LATPOLE, following wcslib's celset/sphs2x conventions.  Pinned against
astropy 4.3.1 / wcslib by tests/test_astro_golden.py (<= 1.2e-9 px, identical
pixel ids); the device path receives the pixel ids computed here.

Also: J2000 equatorial -> galactic (the healpy Rotator(coord=['C','G']) the
reference applies for GLON-/GLAT- maps, COMAPData.py:411-415).
"""
from __future__ import annotations

import numpy as np

D2R = np.pi / 180.0
R2D = 180.0 / np.pi

# J2000 equatorial -> galactic rotation matrix (Hipparcos / healpy convention)
_EQ2GAL = np.array([[-0.0548755604162154, -0.8734370902348850, -0.4838350155487132],
                    [+0.4941094278755837, -0.4448296299600112, +0.7469822444972189],
                    [-0.8676661490190047, -0.1980763734312015, +0.4559837761750669]])


def equatorial_to_galactic(ra, dec):
    ra = np.asarray(ra, dtype=np.float64) * D2R
    dec = np.asarray(dec, dtype=np.float64) * D2R
    v = np.stack([np.cos(dec) * np.cos(ra), np.cos(dec) * np.sin(ra), np.sin(dec)])
    g = np.tensordot(_EQ2GAL, v, axes=1)
    l = np.arctan2(g[1], g[0]) * R2D
    b = np.arcsin(np.clip(g[2], -1, 1)) * R2D
    return np.mod(l, 360.0), b


class CelestialWCS:
    """2-axis celestial WCS: ctype 'XXXX-PRJ' with PRJ in {CAR, SIN, TAN}."""

    def __init__(self, crval, cdelt, crpix, ctype, lonpole=None, latpole=90.0):
        self.crval = np.asarray(crval, dtype=np.float64)
        self.cdelt = np.asarray(cdelt, dtype=np.float64)
        self.crpix = np.asarray(crpix, dtype=np.float64)
        self.ctype = list(ctype)
        self.proj = self.ctype[0][-3:]
        if self.proj not in ('CAR', 'SIN', 'TAN'):
            raise NotImplementedError(f'projection {self.proj} not supported')
        self.galactic = self.ctype[0].startswith('GLON')
        phi0, theta0 = (0.0, 0.0) if self.proj == 'CAR' else (0.0, 90.0)
        a0, d0 = self.crval
        if lonpole is None:
            lonpole = 0.0 if d0 >= theta0 else 180.0
        self.phip = lonpole
        if theta0 == 90.0:
            ap, dp = a0, d0
        else:
            cthe0, sthe0 = np.cos(theta0 * D2R), np.sin(theta0 * D2R)
            sphip, cphip = np.sin((lonpole - phi0) * D2R), np.cos((lonpole - phi0) * D2R)
            x = cthe0 * cphip
            y = sthe0
            z = np.hypot(x, y)
            u = np.arctan2(y, x) * R2D
            v = np.arccos(np.clip(np.sin(d0 * D2R) / z, -1, 1)) * R2D
            cands = []
            for lp in (u + v, u - v):
                if lp > 180:
                    lp -= 360
                elif lp < -180:
                    lp += 360
                if lp > 90:
                    lp = 180 - lp
                elif lp < -90:
                    lp = -180 - lp
                cands.append(lp)
            dp = min(cands, key=lambda lp: abs(lp - latpole))
            zz = np.cos(dp * D2R) * np.cos(d0 * D2R)
            if abs(zz) < 1e-10:      # native pole on a celestial pole: phi(a0) = phi0 fixes ap
                ap = a0 + lonpole - phi0 - 180.0 if dp > 0 else a0 - lonpole + phi0
            else:
                xx = (sthe0 - np.sin(dp * D2R) * np.sin(d0 * D2R)) / zz
                yy = sphip * cthe0 / np.cos(d0 * D2R)
                ap = a0 - np.arctan2(yy, xx) * R2D
        self.eul = (ap, 90.0 - dp, lonpole, np.cos((90.0 - dp) * D2R), np.sin((90.0 - dp) * D2R))
        self.latpole = latpole
        self.wcs = self          # astropy spelling: w.wcs.ctype / w.wcs.cdelt

    def to_header(self):
        """FITS WCS keywords (ordered list of (key, value)) for the map writer."""
        return [('WCSAXES', 2), ('CRPIX1', float(self.crpix[0])), ('CRPIX2', float(self.crpix[1])),
                ('CDELT1', float(self.cdelt[0])), ('CDELT2', float(self.cdelt[1])),
                ('CUNIT1', 'deg'), ('CUNIT2', 'deg'), ('CTYPE1', self.ctype[0]), ('CTYPE2', self.ctype[1]),
                ('CRVAL1', float(self.crval[0])), ('CRVAL2', float(self.crval[1])),
                ('LONPOLE', float(self.phip)), ('LATPOLE', float(self.latpole))]

    def _native(self, lng, lat):
        e0, e1, e2, ce1, se1 = self.eul
        dl = (lng - e0) * D2R
        cl, sl = np.cos(lat * D2R), np.sin(lat * D2R)
        x = sl * se1 - cl * ce1 * np.cos(dl)
        small = np.abs(x) < 1e-5
        if np.any(small):
            x = np.where(small, -np.cos(lat * D2R + e1 * D2R) + cl * ce1 * (1 - np.cos(dl)), x)
        y = -cl * np.sin(dl)
        phi = e2 + np.arctan2(y, x) * R2D
        phi = np.where(phi > 180, phi - 360, np.where(phi < -180, phi + 360, phi))
        z = sl * ce1 + cl * se1 * np.cos(dl)
        theta = np.arcsin(np.clip(z, -1, 1)) * R2D
        return phi, theta

    def wcs_world2pix(self, x, y, origin=0):
        lng, lat = np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)
        phi, theta = self._native(lng, lat)
        if self.proj == 'CAR':
            ix, iy = phi, theta
        else:
            if self.proj == 'SIN':
                r = R2D * np.cos(theta * D2R)
            else:
                r = R2D / np.tan(theta * D2R)
            ix = r * np.sin(phi * D2R)
            iy = -r * np.cos(phi * D2R)
        px = self.crpix[0] + ix / self.cdelt[0] - 1 + origin
        py = self.crpix[1] + iy / self.cdelt[1] - 1 + origin
        return px, py


def transform_to_1d(x, y, wcs, nx, ny):
    """COMAPData.transform_to_1d (COMAPData.py:83-117): floor(p + 0.5),
    off-map -> -1, index = py * nx + px."""
    px, py = wcs.wcs_world2pix(x, y, 0)
    px = np.floor(px + 0.5).astype(float)
    py = np.floor(py + 0.5).astype(float)
    px[(px < 0) | (px > nx - 1)] = np.nan
    py[(py < 0) | (py > ny - 1)] = np.nan
    idx = py * nx + px
    idx[np.isnan(idx)] = -1
    return idx.astype(int)
