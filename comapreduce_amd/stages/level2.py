"""Level-2 QA stage (drop-in for comancpipeline/Analysis/Level2Data.py:224-329).

``Level2FitPowerSpectrum`` -- per (feed <= 19, band, scan) of
``averaged_tod/tod``: power spectrum |fft|^2/n at f > 0, narrow lines masked
by three find_peaks / peak_widths passes above 100 auto_rms^2 (f > 0.5 Hz),
then a 30-bin log-binned red-noise fit from 0.05 Hz (PowerSpectra.py).  The
spectra of every (feed, band, scan) come from one device call
(``tools.powerspectra.power_spectra``); peak masking and the L-BFGS-B fit are
host SciPy, as in the reference.  Diagnostic PNGs are not produced.
Outputs ``fnoise_fits/fnoise_fit_parameters`` [20, B, S, 3] and
``fnoise_fits/auto_rms`` [20, B, S] (N_FEEDS = 20 rows, as the reference).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
from scipy.signal import find_peaks, peak_widths

from ..pipeline.datahandling import CALIBRATOR_LIST, COMAPLevel2, to_host
from ..pipeline.running import PipelineFunction
from ..tools.powerspectra import FitPowerSpectrum, positive_freqs, power_spectra


def mask_lines(freqs, power_spectrum, auto_rms, niter=3):
    """Level2Data.py:288-299: drop [left_ips, right_ips) around each peak above 100 auto_rms^2."""
    mask = np.ones(freqs.size, dtype=bool)
    indices = np.arange(freqs.size, dtype=int)
    for _ in range(niter):
        select = mask & (freqs > 0.5)
        peak_idx, _ = find_peaks(power_spectrum[select], height=auto_rms ** 2 * 100, distance=100)
        peak_idx = indices[select][peak_idx]
        _, _, left_ips, right_ips = peak_widths(power_spectrum, peak_idx, rel_height=0.85)
        for i in range(len(peak_idx)):
            mask[int(left_ips[i]):int(right_ips[i])] = False
    return mask


@dataclass
class Level2FitPowerSpectrum(PipelineFunction):
    name: str = 'Level2FitPowerSpectrum'
    groups: list = field(default_factory=lambda: ['fnoise_fits'])
    source = 'none'
    figure_directory: str = 'figures'
    _full_figure_directory: str = 'figures'
    N_FEEDS: int = 20
    N_BANDS: int = 4
    SAMPLE_RATE: float = 50.
    N_CHANNELS: int = 1024
    STATE: bool = True
    overwrite: bool = False
    device: int = None      # None: torch's current device (LOCAL_RANK under torchrun)
    data: dict = field(default_factory=dict)

    @property
    def save_data(self):
        return self.data, {}

    def __call__(self, data, level2_data: COMAPLevel2 = None):
        level2_data = level2_data if level2_data is not None else self.level2
        if data.source_name in CALIBRATOR_LIST:
            return self.STATE
        self._full_figure_directory = f'{self.figure_directory}/{data.obsid}'
        self.run(data, level2_data)
        return self.STATE

    def run(self, data, level2_data):
        edges = np.asarray(to_host(data.scan_edges), dtype=np.int64).reshape(-1, 2)
        n_scans = len(edges)
        self.data = {'fnoise_fits/fnoise_fit_parameters': np.zeros((self.N_FEEDS, self.N_BANDS, n_scans, 3)),
                     'fnoise_fits/auto_rms': np.zeros((self.N_FEEDS, self.N_BANDS, n_scans))}
        tod_any = level2_data['averaged_tod/tod']
        spectra = power_spectra(tod_any, edges, mode='level2', device=self.device)
        tod = np.asarray(to_host(tod_any))
        freqs = [positive_freqs(e - s, self.SAMPLE_RATE) for s, e in edges]
        par = self.data['fnoise_fits/fnoise_fit_parameters']
        arms = self.data['fnoise_fits/auto_rms']
        for (ifeed, feed), iband in level2_data.tod_loop(bands=True):
            if feed > 19:
                continue
            for iscan, (start, end) in enumerate(edges):
                x = tod[ifeed, iband, start:end]
                if np.nansum(x) == 0:
                    continue
                ps = spectra[iscan][ifeed, iband]
                fr = freqs[iscan]
                auto_rms = np.nanstd(np.diff(x)) / np.sqrt(2)
                mask = mask_lines(fr, ps, auto_rms)
                fit = FitPowerSpectrum(nbins=30)
                fit(fr[mask], ps[mask], errors=None, model=fit.red_noise_model, error_func=fit.log_error,
                    P0=None, min_freq=0.05)
                if fit.result is not None:
                    par[ifeed, iband, iscan] = fit.result.x
                    arms[ifeed, iband, iscan] = auto_rms
