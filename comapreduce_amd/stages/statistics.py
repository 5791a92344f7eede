"""Level-2 statistics stages (drop-in for comancpipeline/Analysis/Statistics.py).

``Spikes`` (Statistics.py:31-105): spike mask of the Level-2 band-averaged
TOD -- per (feed, band) auto-rms of the non-zero samples, per scan a
medfilt(100) high-pass, |x| > 10 rms, each run dilated by fit_spikes' window.
The whole mask is one device call (``comap_spikes``, spikes_kernels.hip).
Its output ``spikes/spike_mask`` zeroes destriper weights (COMAPData.py:332-334).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from .. import _native as N
from ..gpu import _torch, to_device
from ..pipeline.datahandling import CALIBRATOR_LIST, COMAPLevel2, to_host
from ..pipeline.running import PipelineFunction


def spike_mask(tod, scan_edges, medfilt_window=100, step=100, threshold=10.0, device=None):
    """Device spike mask of a Level-2 TOD [F, B, T] (NumPy or CUDA tensor) -> CUDA bool [F, B, T]."""
    torch = _torch()
    device = N.current_device() if device is None else int(device)
    dev = torch.device('cuda', device)
    t = to_device(tod, torch.float64, dev)
    F, B, T = t.shape
    edges = np.ascontiguousarray(np.asarray(to_host(scan_edges), dtype=np.int64).reshape(-1, 2))
    mask = N.device_empty((F, B, T), torch.uint8, dev)
    c = N.ctx(device)
    N.bind_stream(c, dev)
    N.check(N.lib().comap_spikes(c, N.dptr(t), F * B, T, N.hptr(edges, ctypes.c_int64), edges.shape[0],
                                 int(medfilt_window), int(step), float(threshold), N.dptr(mask)), c, 'comap_spikes')
    return mask.bool()


@dataclass
class Spikes(PipelineFunction):
    name: str = 'Spikes'
    overwrite: bool = False
    STATE: bool = True
    MEDIAN_FILTER_STEP: int = 100
    SPIKE_THRESHOLD: float = 10
    device: int = None      # None: torch's current device (LOCAL_RANK under torchrun)
    device_outputs: bool = False
    data: dict = field(default_factory=lambda: {'spikes/spike_mask': np.empty(1)})

    def __post_init__(self):
        self.groups = list(np.unique([s.split('/')[0] for s in self.data.keys()]))

    @property
    def save_data(self):
        return self.data, {}

    def __call__(self, data, level2_data: COMAPLevel2 = None):
        level2_data = level2_data if level2_data is not None else self.level2
        if data.source_name not in CALIBRATOR_LIST:
            self.run_fit_spikes(data, level2_data)
        return self.STATE

    def run_fit_spikes(self, data, level2_data):
        m = spike_mask(level2_data['averaged_tod/tod'], level2_data.scan_edges, self.MEDIAN_FILTER_STEP, 100,
                       self.SPIKE_THRESHOLD, self.device)
        self.data['spikes/spike_mask'] = m if self.device_outputs else m.cpu().numpy()


def _noise_fit(nu, P, model):
    """NoiseStatistics.fit_power_spectrum after power_spectrum (Statistics.py:173-194)."""
    from scipy.optimize import minimize

    def error(p, x, y, sig2, model):
        chi2 = np.sum((np.log(y) - np.log(model([sig2, p[0], p[1]], x))) ** 2)
        if not np.isfinite(chi2):
            return np.inf
        return chi2

    if len(nu) == 0:
        return [np.nan, np.nan, np.nan]
    P0 = [P[np.argmin((nu - 1) ** 2)], -1]
    gd = nu > 0.1
    result = minimize(error, P0, args=(nu[gd], P[gd], P[-1], model), bounds=([0, None], [None, 0]))
    return [P[-1], result.x[0], result.x[1]]


@dataclass
class NoiseStatistics(PipelineFunction):
    """Statistics.NoiseStatistics (Statistics.py:107-224): per (feed, band, scan)
    15-bin log power spectrum of the spike-interpolated Level-2 TOD and a
    white + red power-law fit -> ``noise_statistics/fnoise`` [F, B, S, 3]
    (= [P_bin[-1], sigma_r^2, alpha]).  Spike interpolation and the spectra
    of every series are one device call (``comap_power_spectra``, mode 1);
    binning and the L-BFGS-B fit are host NumPy/SciPy."""
    name: str = 'NoiseStatistics'
    overwrite: bool = False
    STATE: bool = True
    N_FN_PARAMETERS: int = 3
    device: int = None      # None: torch's current device (LOCAL_RANK under torchrun)
    data: dict = field(default_factory=lambda: {'noise_statistics/fnoise': np.empty(1),
                                                'noise_statistics/auto_rms': np.empty(1)})

    def __post_init__(self):
        self.groups = list(np.unique([s.split('/')[0] for s in self.data.keys()]))

    @property
    def save_data(self):
        return self.data, {}

    def __call__(self, data, level2_data: COMAPLevel2 = None):
        level2_data = level2_data if level2_data is not None else self.level2
        if data.source_name not in CALIBRATOR_LIST:
            self.run_fit_noise(data, level2_data)
        return self.STATE

    @staticmethod
    def model(P, x):
        """sigma_w^2 + sigma_r^2 (f / 0.1 Hz)^alpha (Statistics.py:140-150)."""
        return P[0] + P[1] * np.abs(x / 0.1) ** P[2]

    @staticmethod
    def bin_spectrum(nu_pos, ps_pos, n, sample_rate=1. / 50., nbins=15):
        """NoiseStatistics.power_spectrum's binning (Statistics.py:157-171) of the f > 0 half
        (the f <= 0 bins fall below the first edge)."""
        nu_all = np.fft.fftfreq(int(n), d=sample_rate)
        edges = np.logspace(np.log10(np.min(nu_all[1:n // 2])), np.log10(np.max(nu_all)), nbins + 1)
        top = np.histogram(nu_pos, edges, weights=ps_pos)[0]
        bot = np.histogram(nu_pos, edges)[0]
        gd = bot != 0
        P_bin = np.zeros(bot.size) + np.nan
        nu_bin = np.zeros(bot.size) + np.nan
        nu_bin[gd] = np.histogram(nu_pos, edges, weights=nu_pos)[0][gd] / bot[gd]
        P_bin[gd] = top[gd] / bot[gd]
        gd = (bot != 0) & np.isfinite(P_bin) & (nu_bin != 0)
        return nu_bin[gd], P_bin[gd]

    def run_fit_noise(self, data, level2_data):
        from ..tools.powerspectra import positive_freqs, power_spectra
        edges = np.asarray(to_host(level2_data.scan_edges), dtype=np.int64).reshape(-1, 2)
        tod = level2_data.tod
        n_feeds, n_bands, _ = tod.shape
        mask = level2_data['spikes/spike_mask'] if 'spikes/spike_mask' in level2_data.keys() else None
        spectra = power_spectra(tod, edges, mode='noise', spike_mask=mask, device=self.device)
        out = np.zeros((n_feeds, n_bands, len(edges), self.N_FN_PARAMETERS))
        for iscan, (start, end) in enumerate(edges):
            n = int(end - start)
            nu = positive_freqs(n, 50.)
            for ifeed in range(n_feeds):
                for iband in range(n_bands):
                    nb, Pb = self.bin_spectrum(nu, spectra[iscan][ifeed, iband], n)
                    out[ifeed, iband, iscan] = _noise_fit(nb, Pb, self.model)
        self.data['noise_statistics/fnoise'] = out
