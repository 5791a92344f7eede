"""The COMAPData.read_comap_data golden scenario (used by make_golden.py and
the tests): three synthetic Level-2 files and two map definitions.

* obs 12, Field00, feed 3 flagged with bit 2 (skipped), feed 2 with bit 5 (kept)
* obs 13, Field00, a masked (exact-zero) run inside scan 0 of feed 1
* obs 14, TauA (calibrator: tod_original, no median filter)
Selected feeds (1, 2, 3, 4) out of file feeds 1..5.
Cases: (RA---CAR, band 0, gain filter, no calibration, L=50) and
       (GLON-CAR, band 2, calibration with TauA factors, L=100).
"""
from comapreduce_amd import synthetic

FEEDS = [1, 2, 3, 4]
FILES = [(12, 'Field00', {3: 4, 2: 32}), (13, 'Field00', {}), (14, 'TauA', {})]
N_SAMPLES = 24_000
N_FEEDS = 5


def store():
    s, names = {}, []
    for obs, source, bits in FILES:
        data, attrs, fn = synthetic.level2_mapmaking(obs, n_feeds=N_FEEDS, n_samples=N_SAMPLES,
                                                     bad_feed_bits=bits, source=source)
        s[fn] = (data, attrs)
        names.append(fn)
    return s, names


CASES = {
    'car': dict(map=dict(crval=[170.0, 52.0], cdelt=[-1 / 60., 1 / 60.], crpix=[60, 60],
                         ctype=['RA---CAR', 'DEC--CAR'], nxpix=120, nypix=120),
                kw=dict(iband=0, use_gain_filter=True, offset_length=50, calibration=False)),
    'glon': dict(map=dict(crval=[148.0, 60.0], cdelt=[-1 / 30., 1 / 30.], crpix=[60, 45],
                          ctype=['GLON-CAR', 'GLAT-CAR'], nxpix=120, nypix=90),
                 kw=dict(iband=2, use_gain_filter=True, offset_length=100, calibration=True,
                         calibrator='TauA')),
}
OUTPUTS = ('tod', 'weights', 'pointing', 'remapping_array', 'az', 'el', 'ra', 'dec', 'feedid', 'obsids')
STRIDED = ('az', 'el', 'ra', 'dec')   # stored as v[::STRIDE] to keep the fixture small
STRIDE = 37
