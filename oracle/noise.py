"""ORACLE (test infrastructure only): the Level-2 FFT noise QA stages restated
in NumPy/SciPy, checked against goldens the reference itself produced
(tests/golden/make_golden.py --only-noise).

* Level2FitPowerSpectrum.run   (comancpipeline/Analysis/Level2Data.py:265-329)
  with FitPowerSpectrum          (comancpipeline/Analysis/PowerSpectra.py:6-160)
* NoiseStatistics.run_fit_noise (comancpipeline/Analysis/Statistics.py:107-224)

Never imported by the product (comapreduce_amd/); only tests and bench's
cpu_baseline leg use it, as the checker.
"""
import numpy as np
from scipy.optimize import minimize
from scipy.signal import find_peaks, peak_widths

SAMPLE_RATE = 50.0


# ---------------------------------------------------------------- FitPowerSpectrum (PowerSpectra.py)
def bin_power_spectrum(freqs, ps, nbins, min_freq=None, max_freq=None):
    """FitPowerSpectrum.bin_power_spectrum (PowerSpectra.py:20-49)."""
    if min_freq is None:
        min_freq = np.min(freqs)
    if max_freq is None:
        max_freq = np.max(freqs)
    edges = np.logspace(np.log10(min_freq), np.log10(max_freq), nbins + 1)
    top = np.histogram(freqs, edges, weights=ps)[0]
    bot = np.histogram(freqs, edges)[0]
    gd = bot != 0
    P = np.zeros(bot.size) + np.nan
    nu = np.zeros(bot.size) + np.nan
    nu[gd] = np.histogram(freqs, edges, weights=freqs)[0][gd] / bot[gd]
    P[gd] = top[gd] / bot[gd]
    gd = (bot != 0) & np.isfinite(P) & (nu != 0)
    return nu[gd], P[gd]


def red_noise_model(P, f):
    """FitPowerSpectrum.red_noise_model (PowerSpectra.py:64-73)."""
    s_w, s_r, alpha = P
    return s_w ** 2 + s_r ** 2 * np.abs(f / 1) ** alpha


def log_error(P, f, data, err, model):
    """FitPowerSpectrum.log_error (PowerSpectra.py:105-117)."""
    return np.sum((np.log(data) - np.log(model(P, f))) ** 2)


def fit_red_noise(freqs, ps, nbins=30, min_freq=0.05):
    """FitPowerSpectrum.__call__ with red_noise_model / log_error / P0=None
    (PowerSpectra.py:136-160).  Returns (result or None, nu_bin, P_bin)."""
    nu, P = bin_power_spectrum(freqs, ps, nbins, min_freq=min_freq)
    # PowerSpectra.py:145-146 sets result=None for < 3 bins, then minimizes anyway
    idx = np.argmin((nu - 1) ** 2)
    P0 = [P[-1] ** 0.5, P[idx] ** 0.5, np.log(P[0] / P[-1]) / np.log(nu[0] / nu[-1])]
    res = minimize(log_error, P0, method='L-BFGS-B', args=(nu, P, 1, red_noise_model),
                   bounds=[(P0[0] * 0.95, P0[0] * 1.05), (0, None), (-10, 0)])
    return res, nu, P


# ---------------------------------------------------------------- Level2FitPowerSpectrum (Level2Data.py)
def peak_mask(freqs, ps, auto_rms, niter=3):
    """The find_peaks / peak_widths mask loop of Level2FitPowerSpectrum.run (Level2Data.py:288-299)."""
    mask = np.ones(freqs.size, dtype=bool)
    indices = np.arange(freqs.size, dtype=int)
    for _ in range(niter):
        select = mask & (freqs > 0.5)
        pk, _props = find_peaks(ps[select], height=auto_rms ** 2 * 100, distance=100)
        pk = indices[select][pk]
        _w, _h, left, right = peak_widths(ps, pk, rel_height=0.85)
        for i in range(len(pk)):
            mask[int(left[i]):int(right[i])] = False
    return mask


def level2_fit_power_spectrum(tod, scan_edges, feeds, n_feeds_out=20):
    """Level2FitPowerSpectrum.run (Level2Data.py:265-329) on averaged_tod/tod [F, B, T].
    Returns (fnoise_fit_parameters [20, B, S, 3], auto_rms [20, B, S])."""
    F, B, _ = tod.shape
    S = len(scan_edges)
    par = np.zeros((n_feeds_out, B, S, 3))
    arms = np.zeros((n_feeds_out, B, S))
    for ifeed in range(F):
        if feeds[ifeed] > 19:
            continue
        for iband in range(B):
            for iscan, (s, e) in enumerate(scan_edges):
                x = tod[ifeed, iband, s:e]
                if np.nansum(x) == 0:
                    continue
                ps = np.abs(np.fft.fft(x)) ** 2 / x.size
                fr = np.fft.fftfreq(len(x), d=1. / SAMPLE_RATE)
                ps = ps[fr > 0]
                fr = fr[fr > 0]
                a = np.nanstd(np.diff(x)) / np.sqrt(2)
                m = peak_mask(fr, ps, a)
                res, _, _ = fit_red_noise(fr[m], ps[m])
                if res is not None:
                    par[ifeed, iband, iscan] = res.x
                    arms[ifeed, iband, iscan] = a
    return par, arms


# ---------------------------------------------------------------- NoiseStatistics (Statistics.py)
def noise_model(P, x):
    """NoiseStatistics.model (Statistics.py:140-150)."""
    return P[0] + P[1] * np.abs(x / 0.1) ** P[2]


def noise_power_spectrum(tod, sample_rate=1. / 50., nbins=15):
    """NoiseStatistics.power_spectrum (Statistics.py:152-171)."""
    ps = np.abs(np.fft.fft(tod) ** 2)
    nu = np.fft.fftfreq(ps.size, d=sample_rate)
    return bin_power_spectrum_edges(nu, ps, nbins,
                                    np.min(nu[1:ps.size // 2]), np.max(nu))


def bin_power_spectrum_edges(nu, ps, nbins, lo, hi):
    edges = np.logspace(np.log10(lo), np.log10(hi), nbins + 1)
    top = np.histogram(nu, edges, weights=ps)[0]
    bot = np.histogram(nu, edges)[0]
    gd = bot != 0
    P = np.zeros(bot.size) + np.nan
    nb = np.zeros(bot.size) + np.nan
    nb[gd] = np.histogram(nu, edges, weights=nu)[0][gd] / bot[gd]
    P[gd] = top[gd] / bot[gd]
    gd = (bot != 0) & np.isfinite(P) & (nb != 0)
    return nb[gd], P[gd]


def fit_noise_spectrum(nu, P):
    """NoiseStatistics.fit_power_spectrum after power_spectrum (Statistics.py:173-194)."""
    def error(p, x, y, sig2, model):
        chi2 = np.sum((np.log(y) - np.log(model([sig2, p[0], p[1]], x))) ** 2)
        if not np.isfinite(chi2):
            return np.inf
        return chi2
    if len(nu) == 0:
        return [np.nan, np.nan, np.nan]
    P0 = [P[np.argmin((nu - 1) ** 2)], -1]
    gd = nu > 0.1
    r = minimize(error, P0, args=(nu[gd], P[gd], P[-1], noise_model), bounds=([0, None], [None, 0]))
    return [P[-1], r.x[0], r.x[1]]


def interp_spikes(x, spike_mask):
    """The spike interpolation of NoiseStatistics.run_fit_noise (Statistics.py:216-221)."""
    x = x * 1.
    m = spike_mask.astype(bool)
    good = np.where(~m)[0]
    bad = np.where(m)[0]
    x[m] = np.interp(bad, good, x[~m])
    return x


def noise_statistics(tod, scan_edges, spike_mask=None, n_params=3):
    """NoiseStatistics.run_fit_noise (Statistics.py:209-224) -> fnoise [F, B, S, 3]."""
    F, B, _ = tod.shape
    S = len(scan_edges)
    out = np.zeros((F, B, S, n_params))
    for ifeed in range(F):
        for iband in range(B):
            for iscan, (s, e) in enumerate(scan_edges):
                x = tod[ifeed, iband, s:e] * 1.
                if spike_mask is not None:
                    x = interp_spikes(x, spike_mask[ifeed, iband, s:e])
                nu, P = noise_power_spectrum(x)
                out[ifeed, iband, iscan] = fit_noise_spectrum(nu, P)
    return out
