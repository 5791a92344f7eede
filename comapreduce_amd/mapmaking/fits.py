"""Minimal FITS image I/O for the destriper's output maps.

run_destriper.write_map (reference run_destriper.py:19-50) writes, with
astropy.io.fits, a primary HDU holding the destriped map and image
extensions 'Naive', 'Noise' (sqrt(1/weight)) and 'Hits', all
(nypix, nxpix) float64 with the map WCS in every header.  astropy is not in
this image, so this writes the same structure directly: 2880-byte blocks,
80-character cards, big-endian IEEE doubles (BITPIX = -64).
"""
from __future__ import annotations

import numpy as np

BLOCK = 2880


def _card(key, value=None, comment=''):
    if key == 'END':
        return 'END'.ljust(80)
    if isinstance(value, bool):
        v = ('T' if value else 'F').rjust(20)
    elif isinstance(value, (int, np.integer)):
        v = str(int(value)).rjust(20)
    elif isinstance(value, (float, np.floating)):
        s = repr(float(value)).upper()
        if '.' not in s and 'E' not in s and 'N' not in s:
            s += '.0'
        v = s.rjust(20)
    else:
        s = str(value).replace("'", "''")
        v = ("'" + s.ljust(8) + "'").ljust(20)
    c = f'{key:<8}= {v}'
    if comment:
        c += ' / ' + comment
    if len(c) > 80:
        raise ValueError(f'FITS card too long: {c}')
    return c.ljust(80)


def _header_bytes(cards):
    text = ''.join(_card(*c) for c in cards) + _card('END')
    pad = (-len(text)) % BLOCK
    return (text + ' ' * pad).encode('ascii')


def _data_bytes(a):
    b = np.ascontiguousarray(a, dtype='>f8').tobytes()
    return b + b'\0' * ((-len(b)) % BLOCK)


def write_image_hdus(fname, images, wcs_cards=()):
    """images: list of (extname | None, 2-D array); the first is the primary HDU."""
    with open(fname, 'wb') as f:
        for i, (name, img) in enumerate(images):
            img = np.asarray(img, dtype=np.float64)
            ny, nx = img.shape
            if i == 0:
                cards = [('SIMPLE', True), ('BITPIX', -64), ('NAXIS', 2), ('NAXIS1', nx), ('NAXIS2', ny),
                         ('EXTEND', True)]
            else:
                cards = [('XTENSION', 'IMAGE'), ('BITPIX', -64), ('NAXIS', 2), ('NAXIS1', nx), ('NAXIS2', ny),
                         ('PCOUNT', 0), ('GCOUNT', 1)]
            cards += list(wcs_cards)
            if name:
                cards.append(('EXTNAME', name))
            f.write(_header_bytes(cards))
            f.write(_data_bytes(img))


def read_image_hdus(fname):
    """Inverse of write_image_hdus: list of (header dict, 2-D float64 array)."""
    raw = open(fname, 'rb').read()
    out, pos = [], 0
    while pos < len(raw):
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
                        v = v[1:v.rindex("'")].rstrip().replace("''", "'")
                    elif v in ('T', 'F'):
                        v = v == 'T'
                    else:
                        v = float(v) if any(ch in v for ch in '.EN') else int(v)
                    hdr[key] = v
            if done:
                break
        nx, ny = hdr['NAXIS1'], hdr['NAXIS2']
        n = nx * ny * 8
        data = np.frombuffer(raw[pos:pos + n], dtype='>f8').reshape(ny, nx).astype(np.float64)
        pos += n + ((-n) % BLOCK)
        out.append((hdr, data))
    return out
