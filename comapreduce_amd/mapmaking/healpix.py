"""HEALPix pixels and partial-sky maps for the destriper's healpix mode.

The reference's healpix path (COMAPData.read_pixels_healpix, COMAPData.py:429-469;
read_comap_data(healpix=True), :507-513, :570-574; run_destriper.main :159-161 and
write_map_healpix, run_destriper.py:53-77) uses healpy's ang2pix (RING ordering)
and write_map(partial=True).  healpy is not in this image (nor in its conda
interpreter), so both are restated here from the published HEALPix scheme
(Gorski et al. 2005, ApJ 622, 759; the HEALPix C++ loc2pix / pix2loc formulae,
including the sin(theta) form near the poles) and healpy's partial-map FITS
layout (a BINTABLE of PIXEL + map columns, INDXSCHM = 'EXPLICIT').  Parity with
healpy is UNPINNED; pix2ang_ring exists for the self-consistency tests.
"""
from __future__ import annotations

import numpy as np

from .fits import BLOCK, _header_bytes

UNSEEN = -1.6375e30            # healpy.UNSEEN
_TWOTHIRD = 2.0 / 3.0


def nside2npix(nside: int) -> int:
    return 12 * int(nside) * int(nside)


def ang2pix(nside, theta, phi):
    """healpy.ang2pix(nside, theta, phi) in the RING scheme (int64 array)."""
    nside = int(nside)
    theta = np.asarray(theta, dtype=np.float64)
    phi = np.asarray(phi, dtype=np.float64)
    shape = np.broadcast(theta, phi).shape
    theta, phi = np.broadcast_to(theta, shape).ravel(), np.broadcast_to(phi, shape).ravel()
    z = np.cos(theta)
    za = np.abs(z)
    # fmodulo(phi / (pi/2), 4) in [0, 4)
    tt = phi / (0.5 * np.pi)
    tt = np.where(tt >= 0, np.where(tt < 4.0, tt, np.fmod(tt, 4.0)), np.fmod(tt, 4.0) + 4.0)
    tt = np.where(tt == 4.0, 0.0, tt)
    npix = nside2npix(nside)
    ncap = 2 * nside * (nside - 1)
    nl4 = 4 * nside
    out = np.empty(theta.size, dtype=np.int64)

    eq = za <= _TWOTHIRD
    if eq.any():
        t1 = nside * (0.5 + tt[eq])
        t2 = nside * z[eq] * 0.75
        jp = np.trunc(t1 - t2).astype(np.int64)        # ascending edge line
        jm = np.trunc(t1 + t2).astype(np.int64)        # descending edge line
        ir = nside + 1 + jp - jm                       # ring number counted from z = 2/3, in 1..2n+1
        kshift = 1 - (ir & 1)
        ip = ((jp + jm - nside + kshift + 1 + 2 * nl4) >> 1) % nl4
        out[eq] = ncap + (ir - 1) * nl4 + ip
    cap = ~eq
    if cap.any():
        zc, tc, thc = z[cap], tt[cap], theta[cap]
        tp = tc - np.trunc(tc)
        # near the poles (theta < 0.01 or > pi - 0.01) the sin(theta) form keeps precision
        have_sth = (thc < 0.01) | (thc > np.pi - 0.01)
        zac = np.abs(zc)
        tmp = np.where((zac < 0.99) | ~have_sth, nside * np.sqrt(3.0 * (1.0 - zac)),
                       nside * np.sin(thc) / np.sqrt((1.0 + zac) / 3.0))
        jp = np.trunc(tp * tmp).astype(np.int64)
        jm = np.trunc((1.0 - tp) * tmp).astype(np.int64)
        ir = jp + jm + 1                               # ring number counted from the closest pole
        ip = np.trunc(tc * ir).astype(np.int64)
        ip = np.mod(ip, 4 * ir)
        out[cap] = np.where(zc > 0, 2 * ir * (ir - 1) + ip, npix - 2 * ir * (ir + 1) + ip)
    return out.reshape(shape)


def pix2ang_ring(nside, pix):
    """(theta, phi) of RING pixel centres (healpy.pix2ang); for the tests."""
    nside = int(nside)
    p = np.asarray(pix, dtype=np.int64).ravel()
    npix = nside2npix(nside)
    ncap = 2 * nside * (nside - 1)
    z = np.empty(p.size)
    phi = np.empty(p.size)
    north = p < ncap
    south = p >= npix - ncap
    eq = ~north & ~south
    if north.any():
        q = p[north]
        iring = ((1 + np.sqrt(1 + 2 * q.astype(np.float64))) // 2).astype(np.int64)
        iring = np.where(2 * iring * (iring - 1) > q, iring - 1, iring)
        iring = np.where(2 * (iring + 1) * iring <= q, iring + 1, iring)
        iphi = q + 1 - 2 * iring * (iring - 1)
        z[north] = 1.0 - iring * iring / (3.0 * nside * nside)
        phi[north] = (iphi - 0.5) * (0.5 * np.pi / iring)
    if eq.any():
        q = p[eq] - ncap
        iring = q // (4 * nside) + nside
        iphi = q % (4 * nside) + 1
        fodd = np.where(((iring + nside) & 1) == 1, 1.0, 0.5)
        z[eq] = (2 * nside - iring) * (2.0 / (3.0 * nside))
        phi[eq] = (iphi - fodd) * (0.5 * np.pi / nside)
    if south.any():
        q = npix - p[south]
        iring = ((1 + np.sqrt(2 * q.astype(np.float64) - 1)) // 2).astype(np.int64)
        iring = np.where(2 * iring * (iring - 1) >= q, iring - 1, iring)
        iring = np.where(2 * (iring + 1) * iring < q, iring + 1, iring)
        iphi = 4 * iring + 1 - (q - 2 * iring * (iring - 1))
        z[south] = -1.0 + iring * iring / (3.0 * nside * nside)
        phi[south] = (iphi - 0.5) * (0.5 * np.pi / iring)
    shape = np.shape(pix)
    return np.arccos(np.clip(z, -1, 1)).reshape(shape), phi.reshape(shape)


def index_replace(array1, array2):
    """COMAPData.index_replace (COMAPData.py:43-58): the position of every value of
    array2 in array1 (array1's values unique)."""
    array1 = np.asarray(array1)
    sort_indices = np.argsort(array1)
    inv = np.empty_like(sort_indices)
    inv[sort_indices] = np.arange(sort_indices.size)
    return inv[np.searchsorted(array1[sort_indices], np.asarray(array2))]


COLUMN_NAMES = ('TEMPERATURE', 'Q_POLARISATION', 'U_POLARISATION')   # healpy's names for 3 maps


def write_map_partial(fname, maps, nside, nest=False, column_names=COLUMN_NAMES):
    """healpy.write_map(fname, maps, partial=True) for a few full-sky f64 maps:
    an empty primary HDU and a BINTABLE of the pixels where the first map is not
    UNSEEN -- PIXEL (int32 'J', or int64 'K' beyond 2^31 pixels) and one 'D'
    column per map -- with PIXTYPE / ORDERING / NSIDE / FIRSTPIX / LASTPIX /
    INDXSCHM = 'EXPLICIT' / OBJECT = 'PARTIAL'."""
    maps = np.atleast_2d(np.asarray(maps, dtype=np.float64))
    npix = nside2npix(nside)
    if maps.shape[1] != npix:
        raise ValueError(f'maps must hold {npix} pixels (nside {nside})')
    good = np.abs(maps[0] - UNSEEN) > 1e-5 * abs(UNSEEN)
    pix = np.nonzero(good)[0]
    pfmt, pdt = ('J', '>i4') if npix < 2 ** 31 else ('K', '>i8')
    names = ['PIXEL'] + list(column_names[:maps.shape[0]])
    rec = np.empty(pix.size, dtype=[('PIXEL', pdt)] + [(n, '>f8') for n in names[1:]])
    rec['PIXEL'] = pix
    for i, n in enumerate(names[1:]):
        rec[n] = maps[i, pix]
    cols = [('TTYPE1', 'PIXEL'), ('TFORM1', pfmt)]
    for i, n in enumerate(names[1:], start=2):
        cols += [(f'TTYPE{i}', n), (f'TFORM{i}', 'D')]
    primary = [('SIMPLE', True), ('BITPIX', 8), ('NAXIS', 0), ('EXTEND', True)]
    table = [('XTENSION', 'BINTABLE'), ('BITPIX', 8), ('NAXIS', 2), ('NAXIS1', rec.dtype.itemsize),
             ('NAXIS2', int(pix.size)), ('PCOUNT', 0), ('GCOUNT', 1), ('TFIELDS', len(names))] + cols + [
        ('PIXTYPE', 'HEALPIX'), ('ORDERING', 'NESTED' if nest else 'RING'), ('EXTNAME', 'xtension'),
        ('NSIDE', int(nside)), ('FIRSTPIX', 0), ('LASTPIX', npix - 1), ('INDXSCHM', 'EXPLICIT'),
        ('OBJECT', 'PARTIAL')]
    data = rec.tobytes()
    with open(fname, 'wb') as f:
        f.write(_header_bytes(primary))
        f.write(_header_bytes(table))
        f.write(data + b'\0' * ((-len(data)) % BLOCK))


def read_map_partial(fname):
    """(header dict, record array) of a file written by write_map_partial."""
    raw = open(fname, 'rb').read()
    pos, hdrs = 0, []
    for _ in range(2):
        hdr = {}
        while True:
            block = raw[pos:pos + BLOCK].decode('ascii')
            pos += BLOCK
            done = False
            for k in range(0, BLOCK, 80):
                card = block[k:k + 80]
                key = card[:8].strip()
                if key == 'END':
                    done = True
                    break
                if card[8:10] == '= ':
                    v = card[10:].split(' / ')[0].strip()
                    if v.startswith("'"):
                        v = v[1:v.rindex("'")].rstrip()
                    elif v in ('T', 'F'):
                        v = v == 'T'
                    else:
                        v = float(v) if any(ch in v for ch in '.EN') else int(v)
                    hdr[key] = v
            if done:
                break
        hdrs.append(hdr)
    h = hdrs[1]
    fmt = {'J': '>i4', 'K': '>i8', 'D': '>f8', 'E': '>f4'}
    dt = [(h[f'TTYPE{i}'], fmt[h[f'TFORM{i}']]) for i in range(1, h['TFIELDS'] + 1)]
    rec = np.frombuffer(raw[pos:pos + h['NAXIS1'] * h['NAXIS2']], dtype=dt)
    return h, rec
