"""Per-rank operator time of the configs[4] field (64 obs x 19 feeds x 180k, 4 bands) under
several rank splits, measured on ONE GPU: every rank's share is built as its own problem
and timed alone (set-up, and ms per CG iteration of the native solve: the rank's compute
without the all-reduces).  Splits: 'obs' = equal observation counts (run_destriper.py's
len // size split, rounds 2-5), and contiguous (obs, feed) series ranges balanced on
entries + kappa x offsets (rankplan.balanced_ranges) for several kappa.  The slowest rank
bounds a sharded CG iteration, so max / mean of the per-rank ms is the balance that
matters.  Usage: python scripts/field_balance_probe.py [world ...] (default 2 4 8)."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from comapreduce_amd import synthetic  # noqa: E402
from comapreduce_amd.mapmaking import rankplan as R  # noqa: E402
from comapreduce_amd.mapmaking.destriper import DeviceDestriper  # noqa: E402

N_OBS, NF, L, NB, NPIX = 64, 19, 50, 4, 480 * 480


def rank_times(series):
    pix, tod, w = synthetic.destriper_inputs_device(0, offset_length=L, device=0, seed=5000, n_bands=NB, series=series)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        prob = DeviceDestriper(pix, tod, w, L, NPIX, device=0, map_shape=(480, 480))
        torch.cuda.synchronize()
        setup = time.perf_counter() - t0
        if rep == 0:
            del prob
    nnz = prob.nnz()[0]
    prob.solve(threshold=0.0, niter=3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    prob.solve(threshold=0.0, niter=20)
    torch.cuda.synchronize()
    it = (time.perf_counter() - t0) / 20
    del prob, pix, tod, w
    torch.cuda.empty_cache()
    return {'series': list(series), 'nnz': int(nnz), 'setup_ms': setup * 1e3, 'ms_per_iter': it * 1e3}


def main():
    worlds = [int(a) for a in sys.argv[1:]] or [2, 4, 8]
    ent, no = synthetic.field_series_work(N_OBS, device=0)
    print(json.dumps({'entries_total': int(ent.sum()), 'offsets_per_series': int(no)}), flush=True)
    for world in worlds:
        splits = {'obs': [(NF * (N_OBS * r // world), NF * (N_OBS * (r + 1) // world)) for r in range(world)]}
        for kappa in (0.0, 3.0, 6.5):
            splits[f'kappa{kappa:g}'] = R.balanced_ranges(np.round(ent + kappa * no).astype(np.int64), world)
        for name, rng in splits.items():
            ranks = [rank_times(s) for s in rng]
            ms = np.array([r['ms_per_iter'] for r in ranks])
            st = np.array([r['setup_ms'] for r in ranks])
            nz = np.array([r['nnz'] for r in ranks], float)
            print(json.dumps({'world': world, 'split': name, 'max_ms_per_iter': ms.max(),
                              'iter_max_over_mean': ms.max() / ms.mean(), 'setup_max_ms': st.max(),
                              'setup_max_over_mean': st.max() / st.mean(), 'nnz_max_over_mean': nz.max() / nz.mean(),
                              'ranks': ranks}), flush=True)


if __name__ == '__main__':
    main()
