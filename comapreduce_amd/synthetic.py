"""Deterministic synthetic COMAP Level-1 observations (host, NumPy).

Implements the input spec of SURVEY.md §8(d): f32 spectrometer TOD of shape
[feed, 4 sidebands, 1024 channels, T] at 50 Hz with a vane event on [500, 1500),
Lissajous scans of >= 14,000 samples separated by 1,000-sample gaps, an airmass
atmosphere 8 K (A - 1.4), a common 1/f gain drift and radiometer white noise.

Every feed is drawn from ``np.random.default_rng(SeedSequence([obs_id, feed]))``
so a feed's data do not depend on which other feeds are generated (sharding
does not change the data).  The Level-1 layout mirrors what
``COMAPLevel1`` reads (reference ``comancpipeline/Analysis/DataHandling.py``):

* ``spectrometer/tod``            f32 [F, 4, 1024, T]
* ``spectrometer/band_average``   f32 [F, 4, T]   (channel nanmean)
* ``spectrometer/features``       f64 [T]         (2**bit, 0 = none)
* ``spectrometer/MJD``            f64 [T]
* ``spectrometer/feeds``          i64 [F]
* ``spectrometer/bands``/``frequency``  f64 [4, 1024]
* ``spectrometer/pixel_pointing/pixel_{ra,dec,az,el}`` f64 [F, T]
* ``hk/antenna0/deTracker/{lissajous_status,utc}``
* ``hk/antenna0/vane/Tvane``
* attrs ``comap`` : obsid, source, comment

This module is data generation only; the reduction itself lives in the HIP
kernels (``comapreduce_amd/csrc``).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass

import numpy as np

SAMPLE_RATE = 50.0
N_BANDS = 4
N_CHANNELS = 1024
VANE_START, VANE_END = 500, 1500
HOT_START, HOT_END = 600, 1000
RAMP = 100
SCAN_START = 1500
SCAN_LEN = 14_000
SCAN_GAP = 1_000
T_VANE_K = 290.0
WHITE_SIGMA = 1.0 / np.sqrt(2e9 / 1024 * (1.0 / SAMPLE_RATE))   # ~5.06e-3
FIELD_RA, FIELD_DEC = 170.0, 52.0


@dataclass
class SyntheticConfig:
    n_feeds: int = 1
    n_samples: int = 30_000
    obs_id: int = 1
    feed_numbers: tuple | None = None     # default 1..n_feeds
    source: str = 'Field00'
    comment: str = 'synthetic lissajous'
    scan_len: int = SCAN_LEN
    scan_gap: int = SCAN_GAP
    min_last: int = 12_500                # a later scan shorter than this is not started

    def feeds(self):
        if self.feed_numbers is not None:
            return np.asarray(self.feed_numbers, dtype=np.int64)
        return np.arange(1, self.n_feeds + 1, dtype=np.int64)


def scan_status(n_samples: int, scan_len: int = SCAN_LEN, scan_gap: int = SCAN_GAP,
                min_last: int = 12_500) -> np.ndarray:
    """Lissajous status (1 inside a scan) per spectrometer sample."""
    status = np.zeros(n_samples, dtype=np.int64)
    s = SCAN_START
    while s < n_samples - 100:
        e = min(s + scan_len, n_samples - 100)
        if e - s < min_last and s != SCAN_START:
            break
        status[s:e] = 1
        s = e + scan_gap
    return status


def features_vector(n_samples: int) -> np.ndarray:
    f = np.full(n_samples, 2.0 ** 5)
    f[:VANE_START] = 0.0
    f[VANE_START:VANE_END] = 2.0 ** 13
    return f


def hot_fraction(n_samples: int) -> np.ndarray:
    """Fraction of the hot load in the beam: ramps in/out around [600,1000)."""
    h = np.zeros(n_samples)
    t = np.arange(n_samples)
    up = (t >= VANE_START) & (t < HOT_START)
    h[up] = (t[up] - VANE_START) / float(HOT_START - VANE_START)
    h[(t >= HOT_START) & (t < HOT_END)] = 1.0
    dn = (t >= HOT_END) & (t < HOT_END + RAMP)
    h[dn] = 1.0 - (t[dn] - HOT_END) / float(RAMP)
    return h


def pointing(n_samples: int, feed: int):
    t = np.arange(n_samples) / SAMPLE_RATE
    fo = 0.02 * (feed - 10)
    el = 47.5 + 7.5 * np.sin(2 * np.pi * t / 300.0 + 0.1 * feed)
    az = 180.0 + 20.0 * np.sin(2 * np.pi * t / 600.0) + fo
    dec = FIELD_DEC + 1.0 * np.sin(2 * np.pi * t / 29.0 + 0.3) + fo
    ra = FIELD_RA + 1.0 * np.sin(2 * np.pi * t / 37.0) / np.cos(np.radians(FIELD_DEC)) + fo
    return ra, dec, az, el


def gain_drift(rng, n_samples: int, sigma: float = 2e-4) -> np.ndarray:
    w = rng.standard_normal(n_samples)
    f = np.fft.rfftfreq(n_samples, d=1.0 / SAMPLE_RATE)
    f[0] = f[1]
    ps = (1.0 / f) ** 1.5
    g = np.fft.irfft(np.fft.rfft(w) * np.sqrt(ps), n=n_samples)
    return g / np.std(g) * sigma


def generate_feed(cfg: SyntheticConfig, feed: int):
    """Returns (tod f32[4,1024,T], tsys, gain, ra, dec, az, el) for one feed."""
    T = cfg.n_samples
    rng = np.random.default_rng(np.random.SeedSequence([cfg.obs_id, int(feed)]))
    tsys = rng.uniform(35.0, 45.0, (N_BANDS, N_CHANNELS))
    gain = 1e6 * rng.uniform(0.9, 1.1, (N_BANDS, N_CHANNELS))
    dg = gain_drift(rng, T)
    ra, dec, az, el = pointing(T, int(feed))
    A = 1.0 / np.sin(np.radians(el))
    atm = 8.0 * (A - 1.4)
    hf = hot_fraction(T)
    vane = (np.arange(T) >= VANE_START) & (np.arange(T) < VANE_END)
    # sky level (K) and multiplicative gain drift per sample; the vane region
    # sees the load, no atmosphere/drift
    level = np.where(vane, 0.0, atm)
    mult = np.where(vane, 1.0, 1.0 + dg)
    hot_add = hf * (T_VANE_K - 2.73)
    tod = np.empty((N_BANDS, N_CHANNELS, T), dtype=np.float32)
    for b in range(N_BANDS):
        noise = rng.standard_normal((N_CHANNELS, T), dtype=np.float32) * np.float32(WHITE_SIGMA)
        sig = (tsys[b, :, None] + level[None, :] + hot_add[None, :]) * mult[None, :]
        tod[b] = (gain[b, :, None] * sig * (1.0 + noise)).astype(np.float32)
    return tod, tsys, gain, ra, dec, az, el


def generate_level1(cfg: SyntheticConfig) -> dict:
    """Returns {'data': {path: array}, 'attrs': {path: {k: v}}, 'truth': {...}}."""
    T = cfg.n_samples
    feeds = cfg.feeds()
    F = feeds.size
    tod = np.empty((F, N_BANDS, N_CHANNELS, T), dtype=np.float32)
    pix = {k: np.empty((F, T)) for k in ('ra', 'dec', 'az', 'el')}
    tsys_t = np.empty((F, N_BANDS, N_CHANNELS))
    gain_t = np.empty((F, N_BANDS, N_CHANNELS))
    for i, feed in enumerate(feeds):
        tod[i], tsys_t[i], gain_t[i], pix['ra'][i], pix['dec'][i], pix['az'][i], pix['el'][i] = \
            generate_feed(cfg, int(feed))
    band_average = np.nanmean(tod, axis=2).astype(np.float32)
    mjd = 59000.0 + cfg.obs_id * 0.1 + np.arange(T) / SAMPLE_RATE / 86400.0
    status = scan_status(T, cfg.scan_len, cfg.scan_gap, cfg.min_last)
    # housekeeping sampled half a sample earlier than the spectrometer
    hk_utc = mjd - 0.5 / SAMPLE_RATE / 86400.0
    freq = np.linspace(26.0, 34.0, N_BANDS * N_CHANNELS).reshape(N_BANDS, N_CHANNELS)
    data = {
        'spectrometer/tod': tod,
        'spectrometer/band_average': band_average,
        'spectrometer/features': features_vector(T),
        'spectrometer/MJD': mjd,
        'spectrometer/feeds': feeds,
        'spectrometer/bands': freq.copy(),
        'spectrometer/frequency': freq.copy(),
        'spectrometer/pixel_pointing/pixel_ra': pix['ra'],
        'spectrometer/pixel_pointing/pixel_dec': pix['dec'],
        'spectrometer/pixel_pointing/pixel_az': pix['az'],
        'spectrometer/pixel_pointing/pixel_el': pix['el'],
        'hk/antenna0/deTracker/lissajous_status': status,
        'hk/antenna0/deTracker/utc': hk_utc,
        'hk/antenna0/vane/Tvane': np.full(64, (T_VANE_K - 273.15) * 100.0),
    }
    attrs = {'comap': {'obsid': str(cfg.obs_id), 'source': cfg.source, 'comment': cfg.comment}}
    return {'data': data, 'attrs': attrs, 'truth': {'tsys': tsys_t, 'gain': gain_t}}


def level1_metadata(cfg: SyntheticConfig):
    """Everything but the f32 cube, plus the per-sample signal model the device
    generator (comap_synth_tod) turns into the cube:
    returns (data dict without tod/band_average, attrs, level, mult, hot), the
    last three f64 [F, T] (sky level K, multiplicative gain drift, hot-load
    excess K)."""
    T = cfg.n_samples
    feeds = cfg.feeds()
    F = feeds.size
    pix = {k: np.empty((F, T)) for k in ('ra', 'dec', 'az', 'el')}
    level = np.empty((F, T))
    mult = np.empty((F, T))
    t = np.arange(T)
    vane = (t >= VANE_START) & (t < VANE_END)
    hot = np.broadcast_to(hot_fraction(T) * (T_VANE_K - 2.73), (F, T)).copy()
    for i, feed in enumerate(feeds):
        rng = np.random.default_rng(np.random.SeedSequence([cfg.obs_id, int(feed), 99]))
        pix['ra'][i], pix['dec'][i], pix['az'][i], pix['el'][i] = pointing(T, int(feed))
        A = 1.0 / np.sin(np.radians(pix['el'][i]))
        level[i] = np.where(vane, 0.0, 8.0 * (A - 1.4))
        mult[i] = np.where(vane, 1.0, 1.0 + gain_drift(rng, T))
    mjd = 59000.0 + cfg.obs_id * 0.1 + t / SAMPLE_RATE / 86400.0
    freq = np.linspace(26.0, 34.0, N_BANDS * N_CHANNELS).reshape(N_BANDS, N_CHANNELS)
    data = {
        'spectrometer/features': features_vector(T),
        'spectrometer/MJD': mjd,
        'spectrometer/feeds': feeds,
        'spectrometer/bands': freq.copy(),
        'spectrometer/frequency': freq.copy(),
        'spectrometer/pixel_pointing/pixel_ra': pix['ra'],
        'spectrometer/pixel_pointing/pixel_dec': pix['dec'],
        'spectrometer/pixel_pointing/pixel_az': pix['az'],
        'spectrometer/pixel_pointing/pixel_el': pix['el'],
        'hk/antenna0/deTracker/lissajous_status': scan_status(T, cfg.scan_len, cfg.scan_gap, cfg.min_last),
        'hk/antenna0/deTracker/utc': mjd - 0.5 / SAMPLE_RATE / 86400.0,
        'hk/antenna0/vane/Tvane': np.full(64, (T_VANE_K - 273.15) * 100.0),
    }
    attrs = {'comap': {'obsid': str(cfg.obs_id), 'source': cfg.source, 'comment': cfg.comment}}
    return data, attrs, level, mult, hot


def sha256(arr: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(arr).tobytes()).hexdigest()


# ---------------------------------------------------------------- destriper
def destriper_inputs(n_feeds: int = 2, n_samples: int = 20_000, npix_side: int = 60,
                     offset_length: int = 50, seed: int = 7, offmap_fraction: float = 0.01):
    """Small synthetic destriper problem (pointing int64, tod f64, weights f64).

    1/f offsets + sky + white noise per feed, Lissajous pointing on an
    npix_side x npix_side grid; a fraction of samples is off-map (pixel -1) to
    exercise the m[-1] quirk of op_Z (reference Destriper.py:206-213).
    """
    rng = np.random.default_rng(seed)
    N = n_feeds * n_samples
    t = np.arange(n_samples) / SAMPLE_RATE
    sky = rng.standard_normal((npix_side, npix_side)).cumsum(0).cumsum(1) * 1e-2
    pointing = np.empty(N, dtype=np.int64)
    tod = np.empty(N)
    for f in range(n_feeds):
        x = 0.5 + 0.45 * np.sin(2 * np.pi * t / 23.0 + f)
        y = 0.5 + 0.45 * np.sin(2 * np.pi * t / 31.0 + 2 * f)
        ix = np.clip((x * npix_side).astype(int), 0, npix_side - 1)
        iy = np.clip((y * npix_side).astype(int), 0, npix_side - 1)
        p = iy * npix_side + ix
        s = slice(f * n_samples, (f + 1) * n_samples)
        white = rng.standard_normal(n_samples) * 0.1
        drift = np.cumsum(rng.standard_normal(n_samples)) * 0.01
        tod[s] = sky[iy, ix] + drift + white
        pointing[s] = p
    off = rng.random(N) < offmap_fraction
    pointing[off] = -1
    weights = np.full(N, 1.0 / 0.1 ** 2)
    weights[rng.random(N) < 0.02] = 0.0
    return pointing, tod, weights


def scan_edges_from_status(status: np.ndarray) -> np.ndarray:
    """Scan edges with the reference's shared-endpoint convention
    (RepointEdges.get_scan_positions_source, DataHandling.py:205-228)."""
    scans = np.where(status == 1)[0]
    d = np.diff(scans)
    e = scans[np.concatenate(([0], np.where(d > 1)[0], [scans.size - 1]))]
    return np.array([e[:-1], e[1:]]).T.astype(np.int64)


def level2_mapmaking(obs_id: int, n_feeds: int = 19, n_samples: int = 45_000, sky_seed: int = 3,
                     bad_feed_bits: dict | None = None, source: str = 'Field00',
                     calibrator: str = 'TauA'):
    """Synthetic Level-2 file contents for COMAPData.read_comap_data
    (reference MapMaking/COMAPData.py:247-427): returns (datasets, attrs, filename).

    averaged_tod/{tod,tod_original} f64 [F, 4, T] (zero outside scans, a run of
    exact zeros inside one scan to exercise the ``tod == 0`` compaction),
    spikes/spike_mask bool [F, 4, T], pixel pointing, MJD, feeds, and the
    ``comap`` attrs source / bad_observation (indexed by feed number) /
    ``{calibrator}_calibration_factor_band{0..3}``.
    """
    rng = np.random.default_rng(np.random.SeedSequence([obs_id, 7919]))
    sky_rng = np.random.default_rng(sky_seed)
    kx, ky, ph = sky_rng.uniform(0.5, 3.0, 4), sky_rng.uniform(0.5, 3.0, 4), sky_rng.uniform(0, 6.3, 4)
    T = n_samples
    status = scan_status(T)
    edges = scan_edges_from_status(status)
    inscan = np.zeros(T, dtype=bool)
    for s, e in edges:
        inscan[s:e] = True
    t = np.arange(T)
    feeds = np.arange(1, n_feeds + 1, dtype=np.int64)
    ra = np.empty((n_feeds, T)); dec = np.empty_like(ra); az = np.empty_like(ra); el = np.empty_like(ra)
    tod = np.zeros((n_feeds, N_BANDS, T)); tod_orig = np.zeros_like(tod)
    spikes = np.zeros((n_feeds, N_BANDS, T), dtype=bool)
    for i, f in enumerate(feeds):
        r, d, a, e = pointing(T, int(f))
        dr = 0.3 * np.sin(0.7 * obs_id)
        ra[i], dec[i], az[i], el[i] = r + dr, d + 0.2 * np.cos(1.3 * obs_id), a, e
        for b in range(N_BANDS):
            x, y = np.radians(ra[i] - FIELD_RA), np.radians(dec[i] - FIELD_DEC)
            sig = 0.05 * np.sin(kx[b] * 40 * x + ph[b]) * np.cos(ky[b] * 40 * y)
            drift = np.cumsum(rng.standard_normal(T)) * 2e-4
            white = rng.standard_normal(T) * 5e-3
            v = sig + drift + white + 0.01 * b
            tod_orig[i, b] = np.where(inscan, v + 0.1 * np.sin(t / 900.0), 0.0)
            tod[i, b] = np.where(inscan, v, 0.0)
            sp = rng.choice(T, 5, replace=False)
            spikes[i, b, sp] = True
    s0 = edges[0][0] + 3000
    tod[0, :, s0:s0 + 137] = 0.0                     # masked run inside a scan
    bad = np.zeros(20, dtype=np.int64)
    for f, bits in (bad_feed_bits or {}).items():
        bad[f] = bits
    attrs = {'comap': {'source': source, 'obsid': obs_id, 'bad_observation': bad}}
    for b in range(N_BANDS):
        attrs['comap'][f'{calibrator}_calibration_factor_band{b}'] = rng.uniform(0.8, 1.2, 20)
    mjd = 59000.0 + obs_id * 0.1 + t / SAMPLE_RATE / 86400.0
    data = {'averaged_tod/tod': tod, 'averaged_tod/tod_original': tod_orig,
            'averaged_tod/weights': np.ones_like(tod), 'averaged_tod/scan_edges': edges,
            'spikes/spike_mask': spikes, 'spectrometer/feeds': feeds, 'spectrometer/MJD': mjd,
            'spectrometer/pixel_pointing/pixel_ra': ra, 'spectrometer/pixel_pointing/pixel_dec': dec,
            'spectrometer/pixel_pointing/pixel_az': az, 'spectrometer/pixel_pointing/pixel_el': el}
    filename = f'comap-{obs_id:07d}-2020-06-01-000000_Level2Cont.hd5'
    return data, attrs, filename


C5_AMP_DEG = 3.8      # C5 Lissajous half-width: inside the 480 x 1' map's +-4.0 deg (every sample on-map)


def _field_track(o, n_feeds, n, nx, ny, cdelt, dev, amp):
    """Observation o's Lissajous track of destriper_inputs_device: ra / dec offsets (deg) and
    the CAR pixel ids (int32, off-map -1) of its n_feeds x n samples, on device ``dev``."""
    import math
    import torch
    t = torch.arange(n, device=dev, dtype=torch.float64)[None, :]
    k = torch.arange(o * n_feeds, (o + 1) * n_feeds, device=dev, dtype=torch.float64)[:, None]
    ra = amp * torch.sin(2 * math.pi * t / (1250.0 + 7.0 * k) + 0.37 * k)       # degrees from the field centre
    dec = amp * torch.sin(2 * math.pi * t / (1700.0 + 5.0 * k) + 1.1 * k)
    px = torch.floor(-ra / cdelt + (nx / 2 - 1) + 0.5)
    py = torch.floor(dec / cdelt + (ny / 2 - 1) + 0.5)
    ok = (px >= 0) & (px <= nx - 1) & (py >= 0) & (py <= ny - 1)
    pix = torch.where(ok, py * nx + px, torch.full_like(px, -1)).to(torch.int32)
    return ra, dec, pix


def field_series_work(n_obs: int, n_feeds: int = 19, n_samples: int = 180_000, offset_length: int = 50,
                      nx: int = 480, ny: int = 480, cdelt: float = 1.0 / 60.0, device='cpu', amp: float = C5_AMP_DEG):
    """Per (obs, feed) series of destriper_inputs_device's field (series s = obs * n_feeds +
    feed): the (offset, pixel run) pairs of its pointing (rankplan.offset_pixel_runs), i.e.
    the sparse-operator entries a rank holding it takes on, and its offsets.  The track's
    scan periods grow with the series index (1250 + 7 s samples), so later series cross
    fewer pixels per offset.  Pointing only (no tod / noise); ``device``: 'cpu' or a CUDA
    index.  Returns (entries int64 [n_obs * n_feeds], offsets per series)."""
    import torch
    from .mapmaking.rankplan import offset_pixel_runs
    dev = torch.device(device) if isinstance(device, str) else torch.device('cuda', int(device))
    n = n_samples // offset_length * offset_length
    out = np.zeros(n_obs * n_feeds, dtype=np.int64)
    for o in range(n_obs):
        pix = _field_track(o, n_feeds, n, nx, ny, cdelt, dev, amp)[2]
        out[o * n_feeds:(o + 1) * n_feeds] = offset_pixel_runs(pix, offset_length, groups=n_feeds)
    return out, n // offset_length


def destriper_inputs_device(n_obs: int, n_feeds: int = 19, n_samples: int = 180_000, offset_length: int = 50,
                            nx: int = 480, ny: int = 480, cdelt: float = 1.0 / 60.0, device: int = 0, seed: int = 0,
                            n_bands: int = 1, amp: float = C5_AMP_DEG, obs0: int = 0, series=None):
    """Destriper inputs at the SURVEY.md §8(d) C5 scale, generated on the device
    (bench only): observations obs0 .. obs0 + n_obs - 1 of a field, each n_feeds feeds x
    n_samples samples, every (obs, feed) series cut to a multiple of offset_length;
    Lissajous pointing of half-width ``amp`` degrees over an nx x ny CAR field (pixel =
    floor(x + 0.5), off-map -> -1), smooth sky + random-walk (1/f) offsets + white
    noise, inverse-variance weights.  Returns (pixels int32 [N], tod f64, weights f64)
    CUDA tensors; tod / weights are [N] for n_bands = 1, else [n_bands, N] (the same sky
    and pointing, independent offsets and noise per band).  Every observation is drawn
    from its own generator, so a rank generating observations [obs0, obs0 + n) of a
    field gets exactly those observations' samples of the whole field.
    ``series`` = (lo, hi): instead the (obs, feed) series lo .. hi - 1 of the field (series
    s = obs * n_feeds + feed; n_obs / obs0 ignored) -- the same samples as in the whole
    field, for a rank holding a work-balanced range of series (bench.py's field leg).

    The default half-width (3.8 deg on the +-4.0 deg map) keeps every sample on the
    map.  Rounds 2-4 drew 4.2 deg: ~37 % of the samples then fell off the map and, as
    the reference's op_Z does (Destriper.py:206-213), gathered m[-1] in the projection
    without being binned -- a non-symmetric operator on which the (p == pb) BiCG does
    not converge (the round-5 probe)."""
    import torch
    if n_bands > 1:
        pix, t0, w0 = destriper_inputs_device(n_obs, n_feeds, n_samples, offset_length, nx, ny, cdelt, device, seed,
                                              amp=amp, obs0=obs0, series=series)
        tods = torch.empty((n_bands,) + tuple(t0.shape), dtype=torch.float64, device=t0.device)
        ws = torch.empty_like(tods)
        tods[0], ws[0] = t0, w0
        del t0, w0
        for b in range(1, n_bands):
            _, tods[b], ws[b] = destriper_inputs_device(n_obs, n_feeds, n_samples, offset_length, nx, ny, cdelt,
                                                        device, seed + 7919 * b, amp=amp, obs0=obs0, series=series)
        return pix, tods, ws
    dev = torch.device('cuda', device)
    n = n_samples // offset_length * offset_length
    no = n // offset_length
    s_lo, s_hi = (obs0 * n_feeds, (obs0 + n_obs) * n_feeds) if series is None else (int(series[0]), int(series[1]))
    S = s_hi - s_lo
    pix = torch.empty((S, n), dtype=torch.int32, device=dev)
    tod = torch.empty((S, n), dtype=torch.float64, device=dev)
    w = torch.empty((S, n), dtype=torch.float64, device=dev)
    g = torch.Generator(device=dev)
    for o in range(s_lo // n_feeds, (s_hi + n_feeds - 1) // n_feeds):
        g.manual_seed(int(seed) * 1_000_003 + o)
        a, b = max(s_lo, o * n_feeds), min(s_hi, (o + 1) * n_feeds)      # this observation's rows in range
        keep, rows = slice(a - o * n_feeds, b - o * n_feeds), slice(a - s_lo, b - s_lo)
        ra, dec, p = _field_track(o, n_feeds, n, nx, ny, cdelt, dev, amp)
        sky = 0.05 * torch.sin(2.1 * ra) * torch.cos(1.7 * dec)
        steps = torch.randn((n_feeds, no), generator=g, device=dev, dtype=torch.float64) * 2e-3
        sky += torch.cumsum(steps, dim=1).repeat_interleave(offset_length, dim=1)
        sigma = 4e-3 + 2e-3 * torch.rand((n_feeds, 1), generator=g, device=dev, dtype=torch.float64)
        sky += sigma * torch.randn((n_feeds, n), generator=g, device=dev, dtype=torch.float64)
        pix[rows] = p[keep]
        tod[rows] = sky[keep]
        w[rows] = (1.0 / sigma ** 2)[keep]
    return pix.reshape(-1), tod.reshape(-1), w.reshape(-1)
