"""Known-answer fixtures of the reference's running median on NaN input.

Runs the reference's own filter() -- medianFilter.cpp + Mediator.h compiled unmodified
from /root/reference by oracle/Makefile into oracle/_ref/libmedfilt_ref.so -- on seeded
series holding NaN (single samples, runs, head and tail, windows dominated by NaN, all
NaN), +-inf mixed in, even and odd windows (w = 6000 / 400 / 401 / 100 / 6 / 1), series
shorter than the window, and the reflect-padded form COMAPData.median_filter /
Level1Averaging.median_filter use.  With NaN every comparison of Mediator is false, so
the output follows the two-heap's insertion history: the fixtures pin that.

Writes tests/golden/golden_medfilt_nan.npz (inputs x_<name>, outputs y_<name>, windows
w_<name>, reflect flag r_<name>).  Usage: python tests/golden/make_medfilt_nan.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402


def cases():
    rng = np.random.default_rng(2026)

    def base(n):
        return np.round(rng.standard_normal(n), 2)
    out = {}
    x = base(5000); x[1234] = np.nan
    out['single_w400'] = (x, 400, False)
    x = base(5001); x[2000:2300] = np.nan
    out['run300_w401'] = (x, 401, False)
    x = base(3000); x[:5] = np.nan; x[-7:] = np.nan
    out['head_tail_w100'] = (x, 100, False)
    x = base(20000); x[rng.random(20000) < 0.01] = np.nan
    out['scattered_w6000'] = (x, 6000, False)
    x = base(13000); x[4000:8000] = np.nan
    out['run4000_w6000'] = (x, 6000, False)
    x = base(2000); x[rng.random(2000) < 0.03] = np.nan; x[rng.random(2000) < 0.03] = np.inf
    x[rng.random(2000) < 0.03] = -np.inf
    out['mixed_inf_w6'] = (x, 6, False)
    x = base(1000); x[[0, 10, 999]] = np.nan
    out['w1'] = (x, 1, False)
    x = base(300)
    out['short_w400'] = (x, 400, False)
    x = base(300); x[150] = np.nan
    out['short_nan_w401'] = (x, 401, False)
    x = np.full(500, np.nan)
    out['all_nan_w100'] = (x, 100, False)
    x = base(1500); x[700:705] = np.nan; x[0] = np.nan
    out['reflect_w400'] = (x, 400, True)
    x = base(9000); x[rng.random(9000) < 0.002] = np.nan
    out['reflect_w6000'] = (x, 6000, True)
    return out


def main():
    if oracle.ref_lib() is None:
        raise SystemExit('oracle/_ref/libmedfilt_ref.so is not built (make -C oracle, reference present)')
    arrays = {}
    for name, (x, w, reflect) in cases().items():
        if reflect:
            z = np.concatenate((x[::-1], x, x[::-1]))
            y = oracle.medfilt_reference(z, w)[x.size:2 * x.size].copy()
        else:
            y = oracle.medfilt_reference(x.copy(), w)
        arrays[f'x_{name}'] = x
        arrays[f'y_{name}'] = y
        arrays[f'w_{name}'] = np.int64(w)
        arrays[f'r_{name}'] = np.int64(reflect)
    np.savez_compressed(os.path.join(HERE, 'golden_medfilt_nan.npz'), **arrays)
    print('wrote', len(arrays) // 4, 'cases')


if __name__ == '__main__':
    main()
