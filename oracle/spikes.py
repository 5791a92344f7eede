"""ORACLE (test infrastructure only): Statistics.Spikes restated in NumPy
(comancpipeline/Analysis/Statistics.py:31-105, DataHandling.py:591-597)."""
import numpy as np

from . import medfilt


def tod_auto_rms(row):
    """COMAPLevel2.tod_auto_rms (DataHandling.py:591-597)."""
    t = row[row != 0]
    N = t.size // 2 * 2
    return np.nanstd(t[:N:2] - t[1:N:2]) / np.sqrt(2)


def median_filter(tod, w):
    """Spikes.median_filter (Statistics.py:63-73)."""
    if any(~np.isfinite(tod)):
        return np.zeros(tod.size)
    if tod.size < w:
        return np.zeros(tod.size) + np.nanmedian(tod)
    return medfilt(tod.astype(np.float64), w)[:tod.size]


def fit_spikes(tod, rms, w=100, thr=10.0, step=100):
    """Spikes.fit_spikes (Statistics.py:75-93)."""
    clean = tod - median_filter(tod, w)
    mask = np.abs(clean) > rms * thr
    diff = np.diff(mask.astype(float))
    starts = np.where(diff > 0)[0]
    ends = np.where(diff < 0)[0]
    if mask[0]:
        starts = np.insert(starts, 0, 0)
    if mask[-1]:
        ends = np.append(ends, clean.size)
    for s, e in zip(starts, ends):
        mask[int(max(0, s - step)):int(min(tod.size, e + step))] = True
    return mask


def spike_mask(tod, edges):
    F, B, T = tod.shape
    out = np.zeros((F, B, T), dtype=bool)
    for f in range(F):
        for b in range(B):
            rms = tod_auto_rms(tod[f, b])
            for s, e in edges:
                out[f, b, s:e] = fit_spikes(tod[f, b, s:e], rms)
    return out
