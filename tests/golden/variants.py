"""Edge-case Level-1 observations shared by make_golden.py and the tests.

Each variant is the synthetic generator's output with a deterministic edit:
  nan      NaNs inside the scan: a short burst in a fitted channel (select_time
           drops those samples for the whole band), a partly-NaN fitted
           channel, a fully-NaN unfitted channel, a single NaN sample
           (fill_bad_data / select_time paths, Level1Averaging.py:204, 658-665)
  constel  the scan's features are all 2**9 (constant-elevation: per-channel
           nanmedian atmosphere, Level1Averaging.py:242-244)
  calib    source 'TauA' (calibrator scan edges DataHandling.py:231-245,
           median atmosphere + no gain subtraction, Level1Averaging.py:647-648, 719-724)
  tinyscan two extra Lissajous runs of 2 and 3 samples right after the first scan, so
           scans 1 and 2 are 3 and 4 samples long: fit_power_spectrum raises
           (ValueError / IndexError, Level1Averaging.py:552-589) and dG = None
           (:834-838); the atmosphere fit has < 100 samples (NaN fit)
  f3       3 feeds numbered 1, 2, 20, T = 30,000 (two full scans): multi-feed unit
           tables, per-feed gain weights, and the feeds > 19 skip (:817-818)
  inf      +-inf Level-1 samples, T = 30,000 (two scans), all in scan 0 at even
           stride-4 positions, so normalise_data's rms of those channels is NaN
           (Level1Averaging.py:667-679) and their filtered rows are NaN: the
           fit_power_spectrum gate passes (nanmean skips them, :571), b = P^T Z d is
           non-finite, cg's matvec raises and solve_gain_solution returns dG = 0
           (GainSubtraction.py:127-128, 154-158); scan 1 keeps its gain fit
  infodd   +inf / -inf samples at odd stride-4 positions (finite rms): the regression
           of the median filter (np.linalg.solve, :701-705) turns the row into a mix
           of +-inf and NaN, the band-0 channel nanmean holds +-inf so the gate raises
           (dG = None, :834-838), and the band averages keep the +-inf entries
           (only NaN becomes 0, :596-597)
"""
import numpy as np

from comapreduce_amd import synthetic

T_EDGE = 16_000


def make(name):
    if name == 'f3':
        return synthetic.generate_level1(synthetic.SyntheticConfig(**F3_CONFIG))
    if name == 'calib':
        cfg = synthetic.SyntheticConfig(n_feeds=1, n_samples=T_EDGE, obs_id=11, source='TauA')
    else:
        cfg = synthetic.SyntheticConfig(n_feeds=1, n_samples=30_000 if name == 'inf' else T_EDGE,
                                        obs_id={'nan': 12, 'constel': 13, 'tinyscan': 14, 'inf': 16,
                                                'infodd': 15}[name])
    gen = synthetic.generate_level1(cfg)
    d = gen['data']
    if name == 'nan':
        tod = d['spectrometer/tod']
        tod[0, 0, 100, 3000:3010] = np.nan      # fitted channel: 10 samples leave select_time (band 0)
        tod[0, 3, 700, 8000:8050] = np.nan      # fitted channel, band 3
        tod[0, 1, 5, 1500:] = np.nan            # unfitted channel, NaN over the whole scan
        tod[0, 2, 300, 5000] = np.nan           # single sample
        d['spectrometer/band_average'] = np.nanmean(tod, axis=2).astype(np.float32)
    elif name in ('inf', 'infodd'):
        tod = d['spectrometer/tod']
        s0 = synthetic.SCAN_START                  # scan 0 = [1500, 15499)
        if name == 'inf':
            tod[0, 0, 100, s0 + 1500] = np.inf         # offset = 0 mod 4: in tod[..., 0::4]
            tod[0, 2, 300, s0 + 3502] = -np.inf        # offset = 2 mod 4: in tod[..., 2::4]
            tod[0, 1, 200, s0 + 2500:s0 + 2505] = np.inf
        else:
            tod[0, 0, 100, s0 + 1501] = np.inf         # offset = 1 mod 4
            tod[0, 1, 300, s0 + 1503] = -np.inf        # offset = 3 mod 4
        d['spectrometer/band_average'] = np.nanmean(tod, axis=2).astype(np.float32)
    elif name == 'constel':
        f = d['spectrometer/features']
        f[synthetic.SCAN_START:] = 2.0 ** 9
    elif name == 'tinyscan':
        st = d['hk/antenna0/deTracker/lissajous_status']
        e0 = synthetic.SCAN_START + synthetic.SCAN_LEN       # first run is [1500, 15500)
        st[e0 + 1:e0 + 3] = 1                                # run of 2 -> scan of 3 samples
        st[e0 + 4:e0 + 7] = 1                                # run of 3 -> scan of 4 samples
    return gen


F3_CONFIG = dict(n_feeds=3, n_samples=30_000, obs_id=5, feed_numbers=(1, 2, 20))
F3_STRIDE = 7          # the f3 golden keeps averaged_tod/* at every 7th sample (fixture size)
NAMES = ('nan', 'constel', 'calib', 'tinyscan', 'f3', 'inf', 'infodd')


def spikes_level2(golden_dir):
    """Level-2 input of the Spikes golden: the C1 golden averaged_tod with
    injected spikes (single samples, a 3-sample burst, one at a scan edge,
    one at the first sample of the file) and one scan-band with a NaN."""
    import os
    g = np.load(os.path.join(golden_dir, 'golden_l1_c1.npz'))
    tod = g['averaged_tod__tod'].copy()
    edges = g['averaged_tod__scan_edges']
    tod[0, 0, 5000] += 3.0
    tod[0, 1, 9000:9003] -= 2.5
    tod[0, 2, edges[0, 0]] += 4.0
    tod[0, 3, 20000] += 1.0
    tod[0, 3, 25000] = np.nan
    return tod, edges


def noise_level2(golden_dir):
    """Level-2 input of the noise-QA goldens (Level2FitPowerSpectrum,
    NoiseStatistics): feed 1 = the C1 golden averaged_tod plus two narrow
    lines (1.7 Hz, 6.3 Hz) so the find_peaks masking runs; feed 20 = a copy
    (skipped by Level2FitPowerSpectrum: feed > 19); one all-zero scan-band
    (nansum == 0 skip).  A spike mask with a few runs, one touching a scan
    edge, for NoiseStatistics' interpolation."""
    import os
    g = np.load(os.path.join(golden_dir, 'golden_l1_c1.npz'))
    one = g['averaged_tod__tod'][0]
    edges = g['averaged_tod__scan_edges']
    T = one.shape[-1]
    t = np.arange(T) / 50.0
    rng = np.random.default_rng(2024)
    tod = np.stack([one, one * 1.3 + 0.01 * rng.standard_normal(one.shape)]).astype(np.float64)
    sd = np.nanstd(np.diff(one, axis=-1))
    tod[0] += sd * (3.0 * np.sin(2 * np.pi * 1.7 * t) + 2.0 * np.sin(2 * np.pi * 6.3 * t + 0.4))
    s1, e1 = edges[1]
    tod[1, 2, s1:e1] = 0.0
    mask = np.zeros(tod.shape, dtype=bool)
    mask[0, 0, 4000:4210] = True
    mask[0, 1, edges[0, 0]:edges[0, 0] + 150] = True
    mask[0, 3, e1 - 120:e1] = True
    mask[1, 1, 12000:12001] = True
    feeds = np.array([1, 20])
    return tod, edges, mask, feeds
