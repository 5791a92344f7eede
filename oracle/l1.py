"""ORACLE (test infrastructure only): Level-1 -> Level-2 reduction restated in NumPy.

Follows comancpipeline v0.9.1 function by function (file:line cited on each),
with the two closed forms verified in SURVEY.md §0 substituted for the sparse
solvers:
  * AtmosphereRemoval.fit_atmosphere's block_diag + spsolve == an independent
    2x2 normal-equation solve per channel (Level1Averaging.py:197-227);
  * gain_subtraction_fit's CG on P^T Z P (== c*I) == dG_t = sum_nu w_nu y_nu,t
    with w = ZP / (P^T Z P) (GainSubtraction.py:17-209).
Every quirk listed in SURVEY.md §8(a) is kept (scan edges that include the gap,
vane event 0 only, the band-mean median filter with an even 6000 window,
in-place zeroing of the gain-masked channels, weight mutation in
weighted_average_over_band, ...).

Never imported by the product package.
"""
import warnings

import numpy as np
from scipy.interpolate import interp1d

from . import medfilt as _medfilt

VANE_BIT = 13
VANE_COLD_TEMP = 2.73
VANE_HOT_TEMP_OFFSET = 273.15
CALIBRATORS = ('TauA', 'CasA', 'CygA', 'jupiter', 'sun', 'saturn', 'moon')  # Tools/Coordinates.py:7-15
MEDFILT_WINDOW = int(50 * 120)   # Level1Averaging.py:833


# ------------------------------------------------------------------ data model
def features(f):
    """COMAPLevel1.features, DataHandling.py:341-349."""
    f = np.array(f) * 1
    good = f != 0
    f[good] = np.log(f[good]) / np.log(2)
    return f.astype(int)


def scan_edges(status, utc, mjd, feats, scan_status_code=1):
    """RepointEdges.get_scan_positions_source, DataHandling.py:205-228."""
    interp = interp1d(utc, status, kind='previous', bounds_error=False,
                      fill_value='extrapolate')(mjd)
    if np.sum(status) == 0:
        select = np.where(feats == 9)[0]
        return np.array([select[0], select[-1]]).reshape(1, 2)
    scans = np.where(interp == scan_status_code)[0]
    d = np.diff(scans)
    edges = scans[np.concatenate(([0], np.where(d > 1)[0], [scans.size - 1]))]
    return np.array([edges[:-1], edges[1:]]).T


def vane_temperature(mjd0, tvane):
    """COMAPLevel1.vane_temperature, DataHandling.py:316-326 (pre-2022 branch:
    MJD 59611 == 2022-02-01)."""
    if mjd0 < 59611.0:
        return np.nanmean(tvane) / 100.0 + VANE_HOT_TEMP_OFFSET
    raise NotImplementedError('post-2022 Tshroud branch not exercised by the oracle')


def airmass(el):
    """COMAPLevel1.airmass, DataHandling.py:398-401."""
    return 1.0 / np.sin(el * np.pi / 180.0)


# ------------------------------------------------------------------ vane
def vane_indices(feats):
    """MeasureSystemTemperature.find_vane_samples, VaneCalibration.py:56-65."""
    flag = feats == VANE_BIT
    idx = np.nonzero(np.diff(flag))[0] + 1
    return idx.reshape((idx.size // 2, 2))


def auto_rms_1d(x):
    """Tools/stats.py:59-72 (1-D branch)."""
    N = (x.size // 2) * 2
    return np.nanstd(x[1:N:2] - x[:N:2]) / np.sqrt(2)


def find_hot_cold(band_average):
    """find_hot_cold_from_tod, VaneCalibration.py:86-141."""
    def find(tod, _rms, greater):
        v = tod * 1.0
        rng = np.nanmax(v) - np.nanmin(v)
        v /= rng
        rms = _rms / rng
        mid = (np.nanmax(v) + np.nanmin(v)) / 2.0
        cmp = np.greater if greater else np.less
        sel = cmp(v - mid, 15 * rms) & (np.abs(np.gradient(v)) < 2e-3)
        return np.arange(v.size, dtype=int)[sel]

    rms = auto_rms_1d(band_average[:, None].ravel())
    # stats.auto_rms on a [N,1] array == the 1-D formula on the column
    hot = find(band_average, rms, True)
    cold = find(band_average, rms, False)
    if len(hot) == 0 or len(cold) == 0:
        return None, None
    hot = np.sort(hot)
    cold = np.sort(cold)
    cold = cold[cold > hot[-1]]
    return hot, cold


def system_temperature_from_tod(t_hot, tod, hot, cold):
    """VaneCalibration.py:67-82 (f32 nanmean, then float64 via the vane temperature)."""
    th = np.nanmean(tod[..., hot], axis=-1)
    tc = np.nanmean(tod[..., cold], axis=-1)
    gain = (th - tc) / (t_hot - VANE_COLD_TEMP)
    return tc / gain, gain


def measure_system_temperature(tod, band_average, feats, t_hot):
    """measure_system_temperature, VaneCalibration.py:143-198 (without PNGs).

    tod f32[F,B,C,T] (host array), band_average f32[F,B,T]."""
    vi = vane_indices(feats)
    nV = vi.shape[0]
    F, B, C, _ = tod.shape
    tsys = np.zeros((nV, F, B, C))
    gain = np.zeros((nV, F, B, C))
    for iv, (s, e) in enumerate(vi):
        for f in range(F):
            for b in range(B):
                hot, cold = find_hot_cold(band_average[f, b, s:e])
                if hot is None or cold is None:
                    continue
                t, g = system_temperature_from_tod(t_hot, np.array(tod[f, b, :, s:e]), hot, cold)
                tsys[iv, f, b] = t
                gain[iv, f, b] = g
    return tsys, gain


# ------------------------------------------------------------------ atmosphere
def atmos_select():
    """Channel set of fit_atmosphere: arange(10,1014) minus the middle five."""
    s = np.arange(10, 1024 - 10, dtype=int)
    return np.delete(s, np.arange(s.size // 2 - 2, s.size // 2 + 3, dtype=int))


def fit_atmosphere(A, tod, minimum_chunk=100):
    """AtmosphereRemoval.fit_atmosphere, Level1Averaging.py:197-227, closed form."""
    sel = atmos_select()
    select_time = np.isfinite(np.sum(tod[sel], axis=0))
    Acut = np.asarray(A, dtype=np.float64)[select_time]
    offset = np.zeros(1024) + np.nan
    atmos = np.zeros(1024) + np.nan
    if Acut.size < minimum_chunk:
        return offset, atmos
    d = tod[sel][:, select_time].astype(np.float64)
    n = float(Acut.size)
    sa = Acut.sum()
    saa = (Acut * Acut).sum()
    sd = d.sum(axis=1)
    sad = d @ Acut
    det = n * saa - sa * sa
    offset[sel] = (saa * sd - sa * sad) / det
    atmos[sel] = (n * sad - sa * sd) / det
    return offset, atmos


def filter_atmosphere(tod, A, edges, feats):
    """AtmosphereRemoval.filter_atmosphere, Level1Averaging.py:229-246."""
    F, B, C, _ = tod.shape
    out = np.zeros((len(edges), F, B, 2, C))
    for f in range(F):
        for b in range(B):
            t = tod[f, b]
            for i, (s, e) in enumerate(edges):
                if np.all(feats[s:e] == 9):
                    out[i, f, b, 0] = np.nanmedian(t[..., s:e], axis=-1)
                    continue
                out[i, f, b] = fit_atmosphere(A[f, s:e], t[..., s:e])
    return out


# ------------------------------------------------------------------ Level1AveragingGainCorrection
def fill_bad_data(tod):
    """Level1Averaging.py:658-665."""
    B, C, n = tod.shape
    r = tod.reshape(B * C, n)
    nan = np.isnan(r)
    if nan.any():
        with warnings.catch_warnings():
            warnings.simplefilter('ignore', RuntimeWarning)
            med = np.nanmedian(r, axis=1)
        r[nan] = (np.ones(r.shape) * med[:, None])[nan]
    return r.reshape(B, C, n)


def remove_atmosphere(A, tod, fit, source=''):
    """remove_atmosphere (Level1Averaging.py:642-656) + subtract_fitted_atmosphere (:188-195)."""
    if source in CALIBRATORS:
        return tod - np.nanmedian(tod, axis=-1)[..., None]
    A = np.asarray(A)
    return tod - (fit[:, 0, :, None] + fit[:, 1, :, None] * A[None, None, :])


def normalise_data(tod):
    """Level1Averaging.py:667-679."""
    dv = 2e9 / 1024.0
    tau = 1.0 / 50.0
    N4 = tod.shape[-1] // 4 * 4
    diff = tod[..., 0:N4:4] - tod[..., 2:N4:4]
    with warnings.catch_warnings():
        warnings.simplefilter('ignore', RuntimeWarning)
        rms = np.nanstd(diff, axis=-1) / np.sqrt(2) * np.sqrt(dv * tau)
    return tod / rms[..., None], rms[..., None]


def median_index():
    idx = np.arange(1024, dtype=int)[10:-10]
    return idx[(idx < 512 - 5) | (idx > 512 + 5)]


def median_filter(tod, w=MEDFILT_WINDOW):
    """Level1AveragingGainCorrection.median_filter, Level1Averaging.py:681-708."""
    B, C, n = tod.shape
    out = np.zeros((B, C, n))
    idx = median_index()
    mf_all = np.full((B, n), np.nan)
    for b in range(B):
        masked = tod[b, idx, :]
        with warnings.catch_warnings():
            warnings.simplefilter('ignore', RuntimeWarning)
            mean = np.nanmean(masked, axis=0)
        if np.nansum(np.isfinite(mean)) < w * 2:
            continue
        pad = np.zeros(3 * n)
        pad[:n] = mean[::-1]
        pad[n:2 * n] = mean
        pad[2 * n:] = mean[::-1]
        mf = _medfilt(pad, w)[n:2 * n]
        mf_all[b] = mf
        A = np.ones((n, 2))
        A[:, 1] = mf
        x = np.linalg.solve(A.T @ A, A.T @ masked.T)
        out[b, idx] = masked - (A @ x).T
    return out, mf_all


def power_spectrum_gate(y0):
    """True when fit_power_spectrum (Level1Averaging.py:552-589) would NOT raise.

    The fit's result is unused (use_prior=False); only its IndexError (no
    finite bins) / ValueError (too few samples) turns dG into None (:834-838)."""
    with warnings.catch_warnings():
        warnings.simplefilter('ignore', RuntimeWarning)
        r = np.nanmean(y0[10:-10], axis=0)
    ps = np.abs(np.fft.fft(r) ** 2)
    nu = np.fft.fftfreq(ps.size, d=1.0 / 50.0)
    if ps.size // 2 <= 1:
        return False
    edges = np.logspace(np.log10(np.min(nu[1:ps.size // 2])), np.log10(np.max(nu)), 16)
    top = np.histogram(nu, edges, weights=ps)[0]
    bot = np.histogram(nu, edges)[0]
    gd = bot != 0
    P = np.full(bot.size, np.nan)
    nub = np.full(bot.size, np.nan)
    nub[gd] = np.histogram(nu, edges, weights=nu)[0][gd] / bot[gd]
    P[gd] = top[gd] / bot[gd]
    gd = (bot != 0) & np.isfinite(P) & (nub != 0)
    return bool(gd.any())


def gain_weights(tsys):
    """Closed form of gain_subtraction_fit + AMatrix + cg (GainSubtraction.py:17-209).

    Returns (w [B*C] or None, bad_values mask [B,C], all_bad).  Raises
    ValueError like AMatrix.z_operation when C = T^T T is not finite."""
    B, C = tsys.shape
    v = np.linspace(-1, 1, 1024 * 4).reshape((4, 1024))
    T = np.ones((B, C, 3))
    with np.errstate(divide='ignore', invalid='ignore'):
        T[..., 0] = 1.0 / tsys
        T[..., 1] = v / tsys
    bad = np.isnan(tsys)
    T[:, :20, :] = 0
    T[:, -20:, :] = 0
    T[:, 507:517, :] = 0
    T[bad, :] = 0
    if bad.sum() == bad.size:
        return None, bad, True
    T = T.reshape(B * C, 3)
    T01 = T[:, :2]
    P = T[:, 2]
    Cm = T01.T @ T01
    if not np.isfinite(np.sum(Cm)):
        raise ValueError('C matrix is not finite in AMatrix.z_operation')
    ZP = P - T01 @ (np.linalg.inv(Cm) @ (T01.T @ P))
    c = P @ ZP
    return ZP / c, bad, False


def gain_subtraction_fit(y, tsys):
    """gain_subtraction_fit, GainSubtraction.py:170-209 -- zeroes y IN PLACE."""
    B, C, n = y.shape
    bad = np.isnan(tsys)
    y[:, :20, :] = 0
    y[:, -20:, :] = 0
    y[:, 507:517, :] = 0
    y[bad, :] = 0
    w, _, all_bad = gain_weights(tsys)
    if all_bad:
        return np.zeros(n)
    if not np.isfinite(y).all():
        # A non-finite y (a NaN / inf sample, or a channel whose normalisation rms is
        # NaN) makes b = P^T Z d non-finite; cg's first matvec on it raises ValueError
        # ('PtZPg is not finite', GainSubtraction.py:127-128), which
        # solve_gain_solution catches and returns g = zeros (:154-158).
        return np.zeros(n)
    return w @ y.reshape(B * C, n)


def weighted_average_over_band(res, wts):
    """Level1Averaging.py:592-599 -- mutates BOTH res (NaN->0) and wts."""
    wts[:, :50] = 0
    wts[:, -50:] = 0
    wts[:, 512] = 0
    wts[np.isnan(res[..., 0])] = 0
    res[np.isnan(res)] = 0
    return np.sum(res * wts[..., None], axis=1) / np.sum(wts[..., None], axis=1)


def auto_rms_rows(tod):
    """Level1AveragingGainCorrection.auto_rms, Level1Averaging.py:512-518."""
    N = tod.shape[-1] // 2 * 2
    with warnings.catch_warnings():
        warnings.simplefilter('ignore', RuntimeWarning)
        return np.nanstd(tod[..., 1:N:2] - tod[..., 0:N:2], axis=-1) / np.sqrt(2)


def reduce_scan(tod_scan, A_scan, fit, tsys, gain, source='', is_first_scan=False):
    """One (feed, scan) of average_tod, Level1Averaging.py:821-867.

    tod_scan f32[4,1024,n] (a copy; fill is applied to it), A_scan [n],
    fit [4,2,1024], tsys/gain [4,1024] (vane event 0).
    Returns (residual_avg [4,n], tod_original [4,n], weights [4]) and a dict of
    intermediates for kernel-level checks."""
    tod_scan = fill_bad_data(tod_scan)
    clean = remove_atmosphere(A_scan, tod_scan, fit, source)
    clean, nf = normalise_data(clean)
    clean, mf = median_filter(clean)
    dG = None
    if power_spectrum_gate(clean[0]) and source not in CALIBRATORS:
        try:
            dG = gain_subtraction_fit(clean, tsys)
        except ValueError:
            dG = None
    with np.errstate(divide='ignore'):
        wts = 1.0 / tsys ** 2
    wts[tsys == 0] = 0
    wts[:, :10] = 0
    wts[:, -10:] = 0
    wts[:, 510:515] = 0
    with np.errstate(divide='ignore', invalid='ignore'):
        if dG is not None:
            res = (clean - dG[None, None, :]) * nf / gain[:, :, None]
        else:
            res = clean * nf / gain[:, :, None]
    res = weighted_average_over_band(res, wts)
    if is_first_scan and dG is not None:
        weighted_average_over_band(clean, wts)      # plotting branch mutates clean & wts
    with np.errstate(invalid='ignore'):
        orig = weighted_average_over_band(clean * tsys[:, :, None], wts)
    weights = 1.0 / auto_rms_rows(res) ** 2
    return res, orig, weights, {'nf': nf, 'mf': mf, 'dG': dG}


def average_tod(tod, A, edges, fit_values, tsys0, gain0, feeds, source=''):
    """Level1AveragingGainCorrection.average_tod, Level1Averaging.py:792-872.

    tod f32[F,4,1024,T]; fit_values [S,F,4,2,1024]; tsys0/gain0 [F,4,1024]."""
    F, B, C, T = tod.shape
    out_tod = np.zeros((F, 4, T))
    out_orig = np.zeros((F, 4, T))
    out_w = np.zeros((F, 4, T))
    for f in range(F):
        if feeds[f] > 19:
            continue
        feed_tod = np.array(tod[f])          # h5py-like fresh copy per feed
        for i, (s, e) in enumerate(edges):
            r, o, w, _ = reduce_scan(feed_tod[..., s:e].copy(), A[f, s:e], fit_values[i, f],
                                     tsys0[f], gain0[f], source, is_first_scan=(i == 0))
            out_tod[f, :, s:e] = r
            out_orig[f, :, s:e] = o
            out_w[f, :, s:e] = w[:, None]
    S = len(edges)
    return {'averaged_tod/tod': out_tod, 'averaged_tod/tod_original': out_orig,
            'averaged_tod/weights': out_w, 'averaged_tod/scan_edges': np.asarray(edges),
            'averaged_tod/frequency_power_spectra': np.zeros((S, F, B, 15, 2)),
            'averaged_tod/frequency_power_spectra_fits': np.zeros((S, F, B, 3))}


def scan_edges_calibrator(feats):
    """RepointEdges.get_scan_positions_calibrator, DataHandling.py:231-245
    (on_source: features not in {13, 0, 16}, :304-307)."""
    idx = np.where((feats != 13) & (feats != 0) & (feats != 16))[0]
    return np.array([[int(min(idx))], [int(max(idx))]]).T


def reduce_level1(data, source=''):
    """Full MeasureSystemTemperature -> AtmosphereRemoval ->
    Level1AveragingGainCorrection on a dict of Level-1 datasets."""
    d = data
    feats = features(d['spectrometer/features'])
    if source in CALIBRATORS:
        edges = scan_edges_calibrator(feats)
    else:
        edges = scan_edges(d['hk/antenna0/deTracker/lissajous_status'], d['hk/antenna0/deTracker/utc'],
                           d['spectrometer/MJD'], feats)
    tod = d['spectrometer/tod']
    t_hot = vane_temperature(d['spectrometer/MJD'][0], d['hk/antenna0/vane/Tvane'])
    tsys, gain = measure_system_temperature(tod, d['spectrometer/band_average'], feats, t_hot)
    A = airmass(d['spectrometer/pixel_pointing/pixel_el'])
    fit = filter_atmosphere(tod, A, edges, feats)
    out = average_tod(tod, A, edges, fit, tsys[0], gain[0], d['spectrometer/feeds'], source)
    out['vane/system_temperature'] = tsys
    out['vane/system_gain'] = gain
    out['atmosphere/fit_values'] = fit
    return out


# ------------------------------------------------------------------ generic channel binning
def level1_averaging(tod, tsys, gain, frequency_bin_size=512):
    """Level1Averaging.average_tod, Level1Averaging.py:292-321 (masks :265-273):
    tod f32 [F, B, C, T]; tsys, gain [F, B, C] (vane event 0).  Same NumPy
    expressions per (feed, band) as the reference."""
    F, B, C, T = tod.shape
    mask = np.zeros(C, dtype=bool)
    mask[:10] = True
    mask[-10:] = True
    mask[511:514] = True
    nlow = C // frequency_bin_size
    avg = np.zeros((F, B, nlow, T))
    sd = np.zeros((F, B, nlow, T))
    for f in range(F):
        for b in range(B):
            x = np.array(tod[f, b])                          # fresh f32 copy (h5py slice)
            x /= gain[f, b, :, None]
            w = (1. / tsys ** 2)[f, b, :, None]
            w[mask, :] = 0
            wsum = np.sum(np.reshape(w, (nlow, frequency_bin_size)), axis=1)
            a = np.sum(np.reshape(x * w, (nlow, frequency_bin_size, T)), axis=1) / wsum[:, None]
            q = np.sum(np.reshape(x ** 2 * w, (nlow, frequency_bin_size, T)), axis=1) / wsum[:, None]
            avg[f, b] = a
            sd[f, b] = np.sqrt(q - a ** 2)
    return avg, sd
