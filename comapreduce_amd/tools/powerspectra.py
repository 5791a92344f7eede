"""Level-2 power spectra on the device + the host-side spectrum fitting.

``power_spectra``   batched positive-frequency power spectra of every
                    (feed, band, scan) of a Level-2 TOD in one device call
                    (``comap_power_spectra``, csrc/spectra_kernels.hip): the
                    np.fft calls of Level2FitPowerSpectrum.run
                    (Analysis/Level2Data.py:275-278, mode 'level2') and of
                    NoiseStatistics.power_spectrum after its spike
                    interpolation (Analysis/Statistics.py:152-156, 216-221,
                    mode 'noise').
``FitPowerSpectrum`` drop-in for comancpipeline/Analysis/PowerSpectra.py:6-160:
                    log-binning and the L-BFGS-B red-noise fit, on the host
                    (30 bins and three parameters: no device work to speak of).
"""
from __future__ import annotations

import ctypes

import numpy as np
from scipy.optimize import minimize

from .. import _native as N
from ..gpu import _torch, to_device
from ..pipeline.datahandling import to_host

MODES = {'level2': 0, 'noise': 1}


def positive_bins(n):
    """Number of np.fft.fftfreq(n) bins > 0: k = 1 .. (n-1)//2."""
    return max((int(n) - 1) // 2, 0)


def power_spectra(tod, scan_edges, mode='level2', spike_mask=None, device=None):
    """Device power spectra of a Level-2 TOD [F, B, T] (NumPy or CUDA tensor).

    Returns one host array per scan, shape [F, B, (n-1)//2] with n the scan
    length: mode 'level2' = |fft(x)|**2 / n, mode 'noise' = |fft(x)**2|, at
    frequencies fftfreq(n, 1/50)[1 : (n-1)//2 + 1] (Hz).  ``spike_mask``
    [F, B, T] (bool) is interpolated over first (NoiseStatistics).
    """
    torch = _torch()
    device = N.current_device() if device is None else int(device)
    dev = torch.device('cuda', device)
    t = to_device(tod, torch.float64, dev)
    F, B, T = t.shape
    edges = np.ascontiguousarray(np.asarray(to_host(scan_edges), dtype=np.int64).reshape(-1, 2))
    nk = np.array([positive_bins(e - s) for s, e in edges], dtype=np.int64)
    offs = np.zeros(len(edges), dtype=np.int64)
    if len(edges):
        offs[1:] = np.cumsum(nk * F * B)[:-1]
    total = int((nk * F * B).sum())
    out = torch.empty(max(total, 1), dtype=torch.float64, device=dev)
    m = None
    if spike_mask is not None:
        m = to_device(spike_mask, torch.uint8, dev)
    c = N.ctx(device)
    N.bind_stream(c, dev)
    N.check(N.lib().comap_power_spectra(c, N.dptr(t), F * B, T, N.hptr(edges, ctypes.c_int64), edges.shape[0],
                                        N.dptr(m) if m is not None else None, MODES[mode],
                                        N.hptr(offs, ctypes.c_int64), N.dptr(out)), c, 'comap_power_spectra')
    host = out.cpu().numpy()
    return [host[o:o + F * B * k].reshape(F, B, k) for o, k in zip(offs, nk)]


def positive_freqs(n, sample_rate=50.0):
    """np.fft.fftfreq(n, d=1/sample_rate)[fftfreq > 0], i.e. bins 1 .. (n-1)//2."""
    f = np.fft.fftfreq(int(n), d=1. / sample_rate)
    return f[1:positive_bins(n) + 1]


class FitPowerSpectrum:
    """comancpipeline/Analysis/PowerSpectra.py:6-160 (same names, arguments and results)."""

    def __init__(self, nbins=15):
        self.nbins = nbins
        self.__result = None

    @property
    def result(self):
        return self.__result

    @result.setter
    def result(self, value):
        self.__result = value

    def bin_power_spectrum(self, freqs, power_spectrum, errors=1, min_freq=None, max_freq=None):
        """Log-spaced bin means of (freqs, power); empty / non-finite bins dropped (PowerSpectra.py:20-49)."""
        if min_freq is None:
            min_freq = np.min(freqs)
        if max_freq is None:
            max_freq = np.max(freqs)
        edges = np.logspace(np.log10(min_freq), np.log10(max_freq), self.nbins + 1)
        top = np.histogram(freqs, edges, weights=power_spectrum)[0]
        bot = np.histogram(freqs, edges)[0]
        gd = bot != 0
        P_bin = np.zeros(bot.size) + np.nan
        nu_bin = np.zeros(bot.size) + np.nan
        nu_bin[gd] = np.histogram(freqs, edges, weights=freqs)[0][gd] / bot[gd]
        P_bin[gd] = top[gd] / bot[gd]
        gd = (bot != 0) & np.isfinite(P_bin) & (nu_bin != 0)
        return nu_bin[gd], P_bin[gd]

    def knee_frequency_model(self, P, freqs):
        sigma_white, knee, alpha = P
        return sigma_white ** 2 * (1 + np.abs(freqs / knee) ** alpha)

    def red_noise_model(self, P, freqs):
        sigma_white, red_noise, alpha = P
        return sigma_white ** 2 + red_noise ** 2 * np.abs(freqs / 1) ** alpha

    def knee_frequency_model_rolloff(self, P, freqs):
        sigma_white, knee, alpha = P
        x = freqs - 0.5
        S = 10 ** (1 - 1 / (1 + np.exp(-x * 10))) / 100. + 0.9
        return sigma_white ** 2 * (1 + np.abs(freqs / knee) ** alpha) * S

    def error(self, P, freqs, data, err, model):
        """PowerSpectra.py:91-103 computes chi2 and returns None (unusable by minimize); kept as is."""
        np.sum((data - model(P, freqs)) ** 2 / err ** 2)

    def log_error(self, P, freqs, data, err, model):
        return np.sum((np.log(data) - np.log(model(P, freqs))) ** 2)

    def __call__(self, freqs, data, errors=None, model=None, error_func=None, P0=None, min_freq=None,
                 max_freq=None):
        if errors is None:
            errors = np.ones_like(data)
        if model is None:
            model = self.knee_frequency_model
        if error_func is None:
            error_func = self.error
        self.nu_bin, self.P_bin = self.bin_power_spectrum(freqs, data, errors, min_freq=min_freq,
                                                          max_freq=max_freq)
        if len(self.nu_bin) < 3:   # PowerSpectra.py:145-146: overwritten by the fit below
            self.result = None
        if P0 is None:
            if model == self.knee_frequency_model:
                P0 = [self.P_bin[-1] ** 0.5, np.mean(self.nu_bin),
                      np.log(self.P_bin[0] / self.P_bin[-1]) / np.log(self.nu_bin[0] / self.nu_bin[-1])]
            elif model == self.red_noise_model:
                idx = np.argmin((self.nu_bin - 1) ** 2)
                P0 = [self.P_bin[-1] ** 0.5, self.P_bin[idx] ** 0.5,
                      np.log(self.P_bin[0] / self.P_bin[-1]) / np.log(self.nu_bin[0] / self.nu_bin[-1])]
        self.result = minimize(error_func, P0, method='L-BFGS-B', args=(self.nu_bin, self.P_bin, 1, model),
                               bounds=[(P0[0] * 0.95, P0[0] * 1.05), (0, None), (-10, 0)])
